// Fused gradient-norm clipping + Adam/AdamW over ONE flat fp32 parameter buffer
// (reference: Lightning gradient_clip_val -> clip_grad_norm_, then
// torch.optim.Adam(lr, weight_decay) with *coupled* L2, src/model.py:150-154, train.py:171).
//
// Two launches replace torch's foreach_norm + foreach_mul + multi-tensor Adam (~10 kernels):
//   1. mta_grad_sqnorm : every workgroup writes the partial sum of (scale*g)^2 of its slice;
//                        workgroup 0 also advances the device-side step counter.
//   2. mta_adam        : every workgroup re-reduces the (<=1024) partials, derives
//                        clip = min(1, max_norm / (||g|| + 1e-6)), and updates its slice.
// lr and step live in device memory, so the step is HIP-graph capturable and the plateau
// scheduler only rewrites one float.  `scale` folds the DDP 1/world_size average in.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace {

constexpr int TPB = 256;

__global__ __launch_bounds__(TPB) void grad_sqnorm_kernel(const float4* __restrict__ g, long n4, float scale,
                                                          float* __restrict__ partials, float* __restrict__ step) {
  __shared__ float scratch[TPB / 64];
  float acc = 0.f;
  for (long i = (long)blockIdx.x * TPB + threadIdx.x; i < n4; i += (long)gridDim.x * TPB) {
    float4 v = g[i];
    v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
    acc = fmaf(v.x, v.x, acc);
    acc = fmaf(v.y, v.y, acc);
    acc = fmaf(v.z, v.z, acc);
    acc = fmaf(v.w, v.w, acc);
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = acc;
    if (blockIdx.x == 0 && step) step[0] += 1.0f;
  }
}

__global__ __launch_bounds__(TPB) void adam_kernel(float4* __restrict__ p, float4* __restrict__ g,
                                                   float4* __restrict__ m, float4* __restrict__ v, long n4,
                                                   const float* __restrict__ partials, int nparts,
                                                   const float* __restrict__ lr_ptr, const float* __restrict__ step_ptr,
                                                   float beta1, float beta2, float eps, float wd, float max_norm,
                                                   float scale, int adamw, float* __restrict__ norm_out,
                                                   float* __restrict__ nonfinite) {
  __shared__ float scratch[TPB / 64];
  float part = 0.f;
  for (int i = threadIdx.x; i < nparts; i += TPB) part += partials[i];
  const float sq = block_sum(part, scratch);
  const float norm = sqrtf(sq);
  float clip = 1.0f;
  if (max_norm > 0.f) clip = fminf(1.0f, max_norm / (norm + 1e-6f));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (norm_out) norm_out[0] = norm;
    if (nonfinite && !isfinite(norm)) nonfinite[0] += 1.0f;  // NaN/Inf guard, read once per epoch
  }
  const float gs = scale * clip;
  const float lr = lr_ptr[0];
  const float t = step_ptr[0];
  const float bc1 = 1.0f - powf(beta1, t);
  const float bc2 = 1.0f - powf(beta2, t);
  const float step_size = lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  const float decay = adamw ? (1.0f - lr * wd) : 1.0f;
  const float l2 = adamw ? 0.0f : wd;
  for (long i = (long)blockIdx.x * TPB + threadIdx.x; i < n4; i += (long)gridDim.x * TPB) {
    float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
    float* pf = reinterpret_cast<float*>(&pp);
    float* gf = reinterpret_cast<float*>(&gg);
    float* mf = reinterpret_cast<float*>(&mm);
    float* vf = reinterpret_cast<float*>(&vv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = gf[k] * gs;
      gf[k] = gk;  // clipped/averaged grad written back (visible to logging / grad-norm hooks)
      gk = fmaf(l2, pf[k], gk);
      mf[k] = fmaf(1.0f - beta1, gk - mf[k], mf[k]);
      vf[k] = fmaf(beta2, vf[k], (1.0f - beta2) * gk * gk);
      const float denom = sqrtf(vf[k]) / bc2_sqrt + eps;
      pf[k] = pf[k] * decay - step_size * (mf[k] / denom);
    }
    p[i] = pp;
    g[i] = gg;
    m[i] = mm;
    v[i] = vv;
  }
}

// ---- single-launch clip + Adam/AdamW (the captured training step's only optimizer node) ----
// Phase 1: every workgroup reduces ||scale*g||^2 over its slice and publishes the partial (write-through
// store, drained, then one agent-scope arrival add on a 64-bit monotonic ticket: the cdna_hip_programming.md
// G16 R1 hand-off, no fences).  Phase 2: every workgroup polls the ticket until the whole grid arrived,
// re-reads the partials in index order (deterministic norm), and updates its slice; with `zero_grad` it
// writes g = 0 back instead of the clipped gradient, which replaces the per-step grad-zeroing fill.
// The grid is capped at one workgroup per CU (256), so every workgroup is co-resident and the poll is
// bounded only for safety (a give-up counts in nonfinite[1]).
constexpr int FUSED_MAX_BLOCKS = 256;
constexpr unsigned FUSED_SPIN_LIMIT = 1u << 22;
// MTA_ADAM_SPIN_LIMIT overrides it (trials time-slicing one GPU wait out another process's slice; a give-up is still
// counted and fails the step); passed as a kernel argument, so it holds on every device and inside captured graphs
inline unsigned fused_spin_limit() {
  static const unsigned v = [] {
    const char* e = getenv("MTA_ADAM_SPIN_LIMIT");
    return (e && atol(e) > 0) ? (unsigned)atol(e) : FUSED_SPIN_LIMIT;
  }();
  return v;
}

// REG: every thread's (at most REG_N) float4 of g, p, m, v are loaded in phase 1, before the grid-wide arrival
// wait, so phase 2 is compute + stores only (the post-barrier HBM round trip of the re-reads was ~1.5 us of a
// ~9 us launch for the 51K-parameter headline model)
constexpr int REG_N = 4;
constexpr int U1 = 8, U2 = 4;  // streaming form: float4 loads in flight per thread (phase 1 / phase 2)
constexpr int STREAM_TPB = TPB;

// Gradient ranges whose producer (a weight-gradient GEMM's split-K reduce, gemm.hip mta_gemm_grad_producer) wrote
// them by overwriting and left the clip-norm partials of them: phase 1 skips them (their squares come from ext, added
// by workgroup b in a fixed order: deterministic), and with zero_grad they are not zeroed (the next step's producer
// overwrites them again).  [s, e) in float4 units.
constexpr int MAX_COVERED = 8;
struct Covered {
  int n;
  long s[MAX_COVERED], e[MAX_COVERED];
  const float* ext;  // producer partials
  int n_ext;
  // ext holds the squares of the WHOLE gradient (world > 1: the xGMI all-reduce's partials of the reduced buffer,
  // csrc/allreduce.hip): phase 1 reads no gradient for the norm; the covered ranges only mark what stays unzeroed
  int ext_only;
};
__device__ __forceinline__ bool covered(const Covered& c, long i) {
  bool in = false;
#pragma unroll
  for (int k = 0; k < MAX_COVERED; ++k) in |= (k < c.n) & (i >= c.s[k]) & (i < c.e[k]);
  return in;
}

// BS threads per workgroup (TPB = 256 for both forms: 1,024-thread workgroups for the streaming form measured slower,
// 93.5 vs 80.8 us at 13.4 M parameters in the mlp_large step, profiles/r5_adam_1024_negative.txt)
template <bool REG, int BS>
__global__ __launch_bounds__(BS) void adam_fused_kernel(float4* __restrict__ p, float4* __restrict__ g,
                                                         float4* __restrict__ m, float4* __restrict__ v, long n4,
                                                         float* __restrict__ partials,
                                                         unsigned long long* __restrict__ ticket,
                                                         const float* __restrict__ lr_ptr, float* __restrict__ step_ptr,
                                                         float beta1, float beta2, float eps, float wd,
                                                         float max_norm, float scale, int adamw, int zero_grad,
                                                         float* __restrict__ norm_out, float* __restrict__ nonfinite,
                                                         unsigned spin_limit, Covered cov) {
  __shared__ float scratch[BS / 64];
  __shared__ float s_norm;
  const long stride = (long)gridDim.x * BS;
  float acc = 0.f;
  float4 rg[REG ? REG_N : 1], rp[REG ? REG_N : 1], rm[REG ? REG_N : 1], rv[REG ? REG_N : 1];
  if constexpr (REG) {
#pragma unroll
    for (int r = 0; r < REG_N; ++r) {
      const long i = (long)blockIdx.x * BS + threadIdx.x + r * stride;
      if (i < n4) {
        rg[r] = g[i];
        rp[r] = p[i];
        rm[r] = m[i];
        rv[r] = v[i];
      } else {
        rg[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int r = 0; r < REG_N; ++r) {
      const long i = (long)blockIdx.x * BS + threadIdx.x + r * stride;
      if (cov.ext_only || (cov.n && covered(cov, i))) continue;
      acc = fmaf(rg[r].x, rg[r].x, acc);
      acc = fmaf(rg[r].y, rg[r].y, acc);
      acc = fmaf(rg[r].z, rg[r].z, acc);
      acc = fmaf(rg[r].w, rg[r].w, acc);
    }
  } else {
    // U1 independent float4 loads in flight per thread: one workgroup per CU (the arrival wait needs them all
    // co-resident) holds too few bytes in flight for HBM with one load per iteration (Little's law)
    for (long i0 = (long)blockIdx.x * BS + threadIdx.x; !cov.ext_only && i0 < n4; i0 += stride * U1) {
      float4 q[U1];
#pragma unroll
      for (int u = 0; u < U1; ++u) {
        const long i = i0 + u * stride;
        q[u] = (i < n4 && !(cov.n && covered(cov, i))) ? g[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U1; ++u) {
        acc = fmaf(q[u].x, q[u].x, acc);
        acc = fmaf(q[u].y, q[u].y, acc);
        acc = fmaf(q[u].z, q[u].z, acc);
        acc = fmaf(q[u].w, q[u].w, acc);
      }
    }
  }
  for (int k = blockIdx.x * BS + threadIdx.x; k < cov.n_ext; k += gridDim.x * BS) acc += cov.ext[k];
  acc = block_sum(acc, scratch) * (scale * scale);
  // the step counter is read by every workgroup BEFORE it arrives (thread 0 loads it and its vmcnt(0) below
  // completes the load before the ticket add; the workgroup reads it from LDS); the last arriver advances it
  __shared__ float s_t;
  if (threadIdx.x == 0) {
    const float t0 = step_ptr[0] + 1.0f;
    s_t = t0;
    __hip_atomic_store(partials + blockIdx.x, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long prev =
        __hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long target = (prev / gridDim.x + 1) * gridDim.x;
    if (prev + 1 == target) step_ptr[0] = t0;
    unsigned long long seen = prev + 1;
    unsigned spins = 0;
    while (seen < target) {
      __builtin_amdgcn_s_sleep(1);
      seen = __hip_atomic_load(ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (++spins > spin_limit) {
        if (nonfinite) atomicAdd(nonfinite + 1, 1.0f);
        break;
      }
    }
  }
  __syncthreads();
  const float t = s_t;
  if (threadIdx.x < 64) {
    // wave 0 reads the partials in parallel (lane b: b, b+64, ...; all loads in flight at once, not a chain of
    // dependent round trips) and reduces them in a fixed order: the same norm on every workgroup and every run
    float sq = 0.f;
    for (int b = threadIdx.x; b < (int)gridDim.x; b += 64)
      sq += __hip_atomic_load(partials + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sq = wave_sum_dpp(sq);
    if (threadIdx.x == 0) s_norm = sqrtf(sq);
  }
  __syncthreads();
  const float norm = s_norm;
  float clip = 1.0f;
  if (max_norm > 0.f) clip = fminf(1.0f, max_norm / (norm + 1e-6f));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (norm_out) norm_out[0] = norm;
    if (nonfinite && !isfinite(norm)) nonfinite[0] += 1.0f;
  }
  const float gs = scale * clip;
  const float lr = lr_ptr[0];
  const float bc1 = 1.0f - powf(beta1, t);
  const float bc2 = 1.0f - powf(beta2, t);
  const float step_size = lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  const float decay = adamw ? (1.0f - lr * wd) : 1.0f;
  const float l2 = adamw ? 0.0f : wd;
  if constexpr (REG) {
#pragma unroll
    for (int r = 0; r < REG_N; ++r) {
      const long i = (long)blockIdx.x * BS + threadIdx.x + r * stride;
      if (i >= n4) continue;
      float4 pp = rp[r], gg = rg[r], mm = rm[r], vv = rv[r];
      float* pf = reinterpret_cast<float*>(&pp);
      float* gf = reinterpret_cast<float*>(&gg);
      float* mf = reinterpret_cast<float*>(&mm);
      float* vf = reinterpret_cast<float*>(&vv);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float gk = gf[k] * gs;
        gf[k] = zero_grad ? 0.0f : gk;
        gk = fmaf(l2, pf[k], gk);
        mf[k] = fmaf(1.0f - beta1, gk - mf[k], mf[k]);
        vf[k] = fmaf(beta2, vf[k], (1.0f - beta2) * gk * gk);
        const float denom = sqrtf(vf[k]) / bc2_sqrt + eps;
        pf[k] = pf[k] * decay - step_size * (mf[k] / denom);
      }
      p[i] = pp;
      if (!(zero_grad && cov.n && covered(cov, i))) g[i] = gg;
      m[i] = mm;
      v[i] = vv;
    }
    return;
  }
  // U2 elements' four streams in flight per thread (same reason as phase 1)
  for (long i0 = (long)blockIdx.x * BS + threadIdx.x; i0 < n4; i0 += stride * U2) {
    float4 pp[U2], gg[U2], mm[U2], vv[U2];
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      const long i = i0 + u * stride;
      if (i < n4) {
        pp[u] = p[i];
        gg[u] = g[i];
        mm[u] = m[i];
        vv[u] = v[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      const long i = i0 + u * stride;
      if (i >= n4) continue;
      float* pf = reinterpret_cast<float*>(&pp[u]);
      float* gf = reinterpret_cast<float*>(&gg[u]);
      float* mf = reinterpret_cast<float*>(&mm[u]);
      float* vf = reinterpret_cast<float*>(&vv[u]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float gk = gf[k] * gs;
        gf[k] = zero_grad ? 0.0f : gk;
        gk = fmaf(l2, pf[k], gk);
        mf[k] = fmaf(1.0f - beta1, gk - mf[k], mf[k]);
        vf[k] = fmaf(beta2, vf[k], (1.0f - beta2) * gk * gk);
        const float denom = sqrtf(vf[k]) / bc2_sqrt + eps;
        pf[k] = pf[k] * decay - step_size * (mf[k] / denom);
      }
      p[i] = pp[u];
      if (!(zero_grad && cov.n && covered(cov, i))) g[i] = gg[u];
      m[i] = mm[u];
      v[i] = vv[u];
    }
  }
}

// register-resident form: one float4 per thread while that fills <= 256 workgroups, at most REG_N
inline bool fused_reg(long n4) { return n4 <= (long)FUSED_MAX_BLOCKS * TPB * REG_N; }
inline int fused_grid_reg(long n4) {
  // one float4 per thread while that fills the grid (fewer, fuller workgroups measured no gain:
  // profiles/r4_adam_reg_per_negative.txt)
  long blocks = (n4 + TPB - 1) / TPB;
  if (blocks < 1) blocks = 1;
  if (blocks > FUSED_MAX_BLOCKS) blocks = FUSED_MAX_BLOCKS;
  return (int)blocks;
}

inline int fused_grid(long n4) {
  long blocks = (n4 + STREAM_TPB * 4 - 1) / (STREAM_TPB * 4);
  if (blocks < 1) blocks = 1;
  if (blocks > FUSED_MAX_BLOCKS) blocks = FUSED_MAX_BLOCKS;
  return (int)blocks;
}

__global__ void scale_kernel(float4* __restrict__ x, long n4, float s) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 a = x[i];
    a.x *= s; a.y *= s; a.z *= s; a.w *= s;
    x[i] = a;
  }
}

inline int grid_for(long n4) {
  long blocks = (n4 + TPB * 4 - 1) / (TPB * 4);  // ~4 float4 per thread
  if (blocks < 1) blocks = 1;
  if (blocks > 1024) blocks = 1024;
  return (int)blocks;
}

}  // namespace

extern "C" int mta_optim_num_partials(long n) { return grid_for(n / 4); }

extern "C" void mta_grad_sqnorm(const float* g, long n, float scale, float* partials, float* step, hipStream_t st) {
  const long n4 = n / 4;
  grad_sqnorm_kernel<<<grid_for(n4), TPB, 0, st>>>(reinterpret_cast<const float4*>(g), n4, scale, partials, step);
}

extern "C" void mta_adam(float* p, float* g, float* m, float* v, long n, const float* partials, const float* lr,
                         const float* step, float beta1, float beta2, float eps, float wd, float max_norm, float scale,
                         int adamw, float* norm_out, float* nonfinite, hipStream_t st) {
  const long n4 = n / 4;
  adam_kernel<<<grid_for(n4), TPB, 0, st>>>(reinterpret_cast<float4*>(p), reinterpret_cast<float4*>(g),
                                            reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v), n4, partials,
                                            grid_for(n4), lr, step, beta1, beta2, eps, wd, max_norm, scale, adamw,
                                            norm_out, nonfinite);
}

// dst[0, bytes) <- 0 as a KERNEL node (a captured hipMemsetAsync node was not ordered against the kernel nodes
// around it on graph replay when several processes share the GPU: profiles/r4_nan_root_cause.txt)
__global__ void zero_bytes_kernel(uint4* __restrict__ dst16, long n16, unsigned char* __restrict__ rest, long nrest) {
  const long stride = (long)gridDim.x * blockDim.x, first = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (long i = first; i < n16; i += stride) dst16[i] = make_uint4(0u, 0u, 0u, 0u);
  for (long i = first; i < nrest; i += stride) rest[i] = 0;
}

extern "C" void mta_zero_bytes(void* dst, long bytes, hipStream_t st) {
  if (bytes <= 0) return;
  const long n16 = ((uintptr_t)dst & 15) ? 0 : bytes / 16;  // unaligned buffers: all bytes one by one
  long blocks = (std::max(n16, bytes - n16 * 16) + 255) / 256;
  blocks = blocks < 1 ? 1 : blocks > 2048 ? 2048 : blocks;
  zero_bytes_kernel<<<(int)blocks, 256, 0, st>>>(reinterpret_cast<uint4*>(dst), n16,
                                                 reinterpret_cast<unsigned char*>(dst) + n16 * 16, bytes - n16 * 16);
}

// dropout seeds += golden-ratio increment (one fresh counter-hash seed per site and step, graph-capturable): the
// 32-true extras' forward has no cast_pad launch that would advance them
__global__ void seeds_advance_kernel(uint64_t* seeds, int n) {
  if ((int)threadIdx.x < n) seeds[threadIdx.x] += 0x9E3779B97F4A7C15ull;
}
extern "C" void mta_seeds_advance(uint64_t* seeds, int n, hipStream_t st) {
  seeds_advance_kernel<<<1, 64, 0, st>>>(seeds, n);
}

extern "C" void mta_scale(float* x, long n, float s, hipStream_t st) {
  const long n4 = n / 4;
  scale_kernel<<<grid_for(n4), TPB, 0, st>>>(reinterpret_cast<float4*>(x), n4, s);
}

extern "C" int mta_adam_fused_partials() { return FUSED_MAX_BLOCKS; }

// ticket: one zero-initialised uint64 per optimizer (monotonic across launches); nonfinite: 2 floats
// ([0] steps with a non-finite norm, [1] arrival waits that gave up)
// covered: n_cov float4 ranges [cov_s[k], cov_e[k]) written by gradient producers, ext: their n_ext norm partials
extern "C" void mta_adam_fused(float* p, float* g, float* m, float* v, long n, float* partials,
                               unsigned long long* ticket, const float* lr, float* step, float beta1, float beta2,
                               float eps, float wd, float max_norm, float scale, int adamw, int zero_grad,
                               float* norm_out, float* nonfinite, int n_cov, const long* cov_s, const long* cov_e,
                               const float* ext, int n_ext, int ext_only, hipStream_t st) {
  const long n4 = n / 4;
  const unsigned spin = fused_spin_limit();
  Covered cov{};
  cov.n = (n_cov < 0 || n_cov > MAX_COVERED) ? 0 : n_cov;  // more ranges than fit: none skipped, ext unused
  for (int k = 0; k < cov.n; ++k) {
    cov.s[k] = cov_s[k];
    cov.e[k] = cov_e[k];
  }
  cov.ext = ext;
  cov.ext_only = ext_only && ext ? 1 : 0;
  cov.n_ext = (cov.n || cov.ext_only) ? n_ext : 0;
  if (fused_reg(n4))
    adam_fused_kernel<true, TPB><<<fused_grid_reg(n4), TPB, 0, st>>>(
        reinterpret_cast<float4*>(p), reinterpret_cast<float4*>(g), reinterpret_cast<float4*>(m),
        reinterpret_cast<float4*>(v), n4, partials, ticket, lr, step, beta1, beta2, eps, wd, max_norm, scale, adamw,
        zero_grad, norm_out, nonfinite, spin, cov);
  else
    adam_fused_kernel<false, STREAM_TPB><<<fused_grid(n4), STREAM_TPB, 0, st>>>(
        reinterpret_cast<float4*>(p), reinterpret_cast<float4*>(g), reinterpret_cast<float4*>(m),
        reinterpret_cast<float4*>(v), n4, partials, ticket, lr, step, beta1, beta2, eps, wd, max_norm, scale, adamw,
        zero_grad, norm_out, nonfinite, spin, cov);
}
