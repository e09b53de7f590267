// Row-wise kernels of the MLP / transformer encoders (BASELINE.json north-star extras):
//
//   mta_cast_pad        fp32 master weights / inputs -> zero-padded bf16 operands (up to 16 tensors, one launch)
//   mta_norm_fwd        LayerNorm or RMSNorm (+ affine, + dropout) of an fp32 row -> bf16 and/or fp32 output,
//                       saving mean / rstd for the backward pass
//   mta_norm_bwd        its backward: dropout mask regenerated from the counter hash, dx (+ residual-stream
//                       gradient) (x GELU'(pre) when the normalised tensor was a GELU output), dgamma / dbeta
//                       reduced per workgroup and added to the fp32 gradient buffer with one atomic per column
//
// One wave per row, VPL float4 per lane (D <= 256 * VPL), rows grid-strided over the workgroup's 4 waves so
// the dgamma/dbeta partials stay in registers until one LDS reduction at the end.
#include "common.h"
#include "cast.h"

#include <type_traits>

namespace {

constexpr int NT_THREADS = 256;

struct CastArgs {
  CastItem item[16];
  int n;
  uint64_t* seeds;  // dropout seeds advanced by this launch (the step's first kernel of the encoder), or null
  int nseeds;
};

__global__ void cast_pad_kernel(CastArgs a) {
  if (blockIdx.x == 0 && blockIdx.y == 0 && (int)threadIdx.x < a.nseeds)
    a.seeds[threadIdx.x] += 0x9E3779B97F4A7C15ull;  // fresh counter-hash seed per step for every dropout site
  cast_item_run(a.item[blockIdx.y], blockIdx.x, gridDim.x);
}

struct NormArgs {
  const float* x;
  const __bf16* xb;     // bf16 x instead of x (wide kernels): the MLP's GELU output stored in bf16
  int ldx;              // row stride of x (elements)
  int M, D, rms;
  float eps;
  const float* gamma;   // [D] or null
  const float* beta;    // [D] or null
  __bf16* y_bf16;       // [M][D]
  float* y_f32;         // [M][D]
  float* mean;          // [M] (LayerNorm)
  float* rstd;          // [M]
  const uint64_t* seed;
  float drop_p;
  // backward
  const float* dy;      // [M][D]
  const __bf16* dyb;    // bf16 dy instead of dy (wide kernels)
  const float* dres;    // [M][ldx] residual-stream gradient added to dx (or null)
  const __bf16* pre;    // [M][D] GELU input: dx *= gelu'(pre) (or null)
  const float* pre_f;   // the same in fp32 (32-true extras; narrow kernels only)
  __bf16* dx_bf16;      // [M][D]
  float* dx_f32;        // [M][ldx]
  float* dgamma;
  float* dbeta;
  float* part;          // per-block partial rows of dgamma / dbeta: [2][blocks][part_ld]
  int part_ld;
  long part_pass;       // floats between the dgamma and dbeta planes
  int gelu_x;           // wide kernels: xb is the bf16 GELU INPUT; the normalised row is gelu(xb) (the MLP's GEMM
                        // then stores only its bf16 pre-activation: no fp32 GELU output written and read back twice)
  // fused alpha / beta heads of the encoder's last layer (wide kernels): forward ab[row] = (h . wa + ba, h . wb + bb)
  // of the normalised row h; backward dy = d_alpha wa + d_beta wb from ab[row] = d(alpha, beta) (rows >= ab_rows: 0)
  // and the head-weight gradients' partial rows (sum over rows of d_alpha h, d_beta h) into hpart
  const float* hw_a;
  const float* hw_b;
  const float* hb_a;
  const float* hb_b;
  float2* ab;
  int ab_rows;
  float* hpart;
};

__device__ __forceinline__ float4 gelu4(float4 v) {
  return make_float4(mta_gelu(v.x), mta_gelu(v.y), mta_gelu(v.z), mta_gelu(v.w));
}

__device__ __forceinline__ float4 ld4(const float* pf, const __bf16* pb, size_t i) {
  if (pb) {
    const bf16x4 b = *reinterpret_cast<const bf16x4*>(pb + i);
    return make_float4((float)b[0], (float)b[1], (float)b[2], (float)b[3]);
  }
  return *reinterpret_cast<const float4*>(pf + i);
}

template <int VPL>
__global__ __launch_bounds__(NT_THREADS) void norm_fwd_kernel(NormArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float invD = 1.0f / (float)a.D;
  // gamma / beta in registers before the row loop: loaded after the row reduction they were a second dependent
  // round trip per row (the transformer's rows are one per wave)
  float4 gm[VPL], bt[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = 4 * (lane + 64 * i);
    gm[i] = (c < a.D && a.gamma) ? *reinterpret_cast<const float4*>(a.gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    bt[i] = (c < a.D && a.beta) ? *reinterpret_cast<const float4*>(a.beta + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int row = blockIdx.x * 4 + wave; row < a.M; row += gridDim.x * 4) {
    float4 v[VPL];
    const float* xr = a.x + (size_t)row * a.ldx;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = 4 * (lane + 64 * i);
      v[i] = c < a.D ? *reinterpret_cast<const float4*>(xr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      s += v[i].x + v[i].y + v[i].z + v[i].w;
    }
    const float mu = a.rms ? 0.f : wave_sum(s) * invD;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = 4 * (lane + 64 * i);
      if (c < a.D) {
        const float dx0 = v[i].x - mu, dx1 = v[i].y - mu, dx2 = v[i].z - mu, dx3 = v[i].w - mu;
        q += dx0 * dx0 + dx1 * dx1 + dx2 * dx2 + dx3 * dx3;
      }
    }
    const float rs = rsqrtf(wave_sum(q) * invD + a.eps);
    if (lane == 0) {
      if (a.mean) a.mean[row] = mu;
      a.rstd[row] = rs;
    }
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = 4 * (lane + 64 * i);
      if (c >= a.D) continue;
      float o[4] = {(v[i].x - mu) * rs * gm[i].x + bt[i].x, (v[i].y - mu) * rs * gm[i].y + bt[i].y,
                    (v[i].z - mu) * rs * gm[i].z + bt[i].z, (v[i].w - mu) * rs * gm[i].w + bt[i].w};
      if (a.seed) {
        float ds4[4];
        mta_dropout_scale4(*a.seed, (uint32_t)row, (uint32_t)c, a.drop_p, ds4);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] *= ds4[j];
      }
      if (a.y_f32) *reinterpret_cast<float4*>(a.y_f32 + (size_t)row * a.D + c) = make_float4(o[0], o[1], o[2], o[3]);
      if (a.y_bf16) {
        bf16x4 b;
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = (__bf16)o[j];
        *reinterpret_cast<bf16x4*>(a.y_bf16 + (size_t)row * a.D + c) = b;
      }
    }
  }
}

// ---- wide rows (D >= 1024: the MLP-large encoder's D = 2048) ----
// One wave per row holds 32+ floats per lane of each operand plus the dgamma/dbeta accumulators (~200 VGPRs,
// 2 waves/SIMD) and pays one dependent round trip per float4 group of gamma/beta/pre/dres interleaved with its
// stores (r2 trace, mlp_large B=64: fwd 61 us, bwd 152 us per call for 78 / 157 MB, 4-5x off the HBM rate).
// Here a 256-thread workgroup spans a row (VPT float4 per thread), every operand of a row is loaded up front
// (the backward also prefetches the NEXT row's operands before reducing the current one), the row sums go
// through one LDS exchange (parity double-buffered: one barrier per row), and each column belongs to exactly
// one thread, so the backward's dgamma/dbeta partials stay in registers and leave as one plain row per block.
// one row's float4 (D-guarded: columns past D read 0), of the input type B16 chosen at compile time -- a runtime
// fp32 / bf16 select around the load made hipcc branch per load and wait for it (the next row's prefetch drained
// before the current row's reductions)
template <bool B16>
__device__ __forceinline__ float4 ld4t(const NormArgs& a, size_t i) {
  if constexpr (B16) {
    const bf16x4 b = *reinterpret_cast<const bf16x4*>(a.xb + i);
    return make_float4((float)b[0], (float)b[1], (float)b[2], (float)b[3]);
  } else {
    return *reinterpret_cast<const float4*>(a.x + i);
  }
}

template <int VPT, bool B16>
__global__ __launch_bounds__(NT_THREADS) void norm_fwd_wide_kernel(NormArgs a) {
  // grid-strided rows (~4 workgroups per CU): gamma / beta loaded once per workgroup instead of once per row, and
  // the next row's loads issued before the current row's reductions (one HBM round trip per row hidden)
  __shared__ float red[2][2][4];  // [row parity][mean / var][wave]
  __shared__ float redh[2][2][4];  // [row parity][alpha / beta][wave] (fused heads)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float invD = 1.0f / (float)a.D;
  const bool heads = a.ab != nullptr;
  float4 gm[VPT], bt[VPT], v[VPT], vn[VPT], wa4[VPT], wb4[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = 4 * (tid + NT_THREADS * i);
    const bool ok = c < a.D;
    gm[i] = (ok && a.gamma) ? *reinterpret_cast<const float4*>(a.gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    bt[i] = (ok && a.beta) ? *reinterpret_cast<const float4*>(a.beta + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    // head weights: slices of the flat parameter buffer (no alignment to rely on)
    wa4[i] = (ok && heads) ? make_float4(a.hw_a[c], a.hw_a[c + 1], a.hw_a[c + 2], a.hw_a[c + 3]) : make_float4(0.f, 0.f, 0.f, 0.f);
    wb4[i] = (ok && heads) ? make_float4(a.hw_b[c], a.hw_b[c + 1], a.hw_b[c + 2], a.hw_b[c + 3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float hba = heads ? a.hb_a[0] : 0.f, hbb = heads ? a.hb_b[0] : 0.f;
  const uint64_t seed = a.seed ? *a.seed : 0ull;
  int row = blockIdx.x;
  if (row >= a.M) return;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = 4 * (tid + NT_THREADS * i);
    v[i] = ld4t<B16>(a, (size_t)row * a.ldx + min(c, a.D - 4));
  }
  for (int it = 0; row < a.M; row += gridDim.x, ++it) {
    const int nrow = row + (int)gridDim.x < a.M ? row + (int)gridDim.x : row;  // clamped: the load is unconditional
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = 4 * (tid + NT_THREADS * i);
      vn[i] = ld4t<B16>(a, (size_t)nrow * a.ldx + min(c, a.D - 4));  // unconditional (clamped column)
    }
    const int par = it & 1;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      if (a.gelu_x) v[i] = gelu4(v[i]);
      if (4 * (tid + NT_THREADS * i) >= a.D) v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    s = wave_sum(s);
    if (lane == 0) red[par][0][wave] = s;
    __syncthreads();
    const float mu = a.rms ? 0.f : ((red[par][0][0] + red[par][0][1]) + (red[par][0][2] + red[par][0][3])) * invD;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      if (4 * (tid + NT_THREADS * i) < a.D) {
        const float d0 = v[i].x - mu, d1 = v[i].y - mu, d2 = v[i].z - mu, d3 = v[i].w - mu;
        q += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
      }
    }
    q = wave_sum(q);
    if (lane == 0) red[par][1][wave] = q;
    __syncthreads();
    const float rs = rsqrtf(((red[par][1][0] + red[par][1][1]) + (red[par][1][2] + red[par][1][3])) * invD + a.eps);
    if (tid == 0) {
      if (a.mean) a.mean[row] = mu;
      a.rstd[row] = rs;
    }
    float pa = 0.f, pb = 0.f;  // fused heads: this thread's share of h . wa, h . wb
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = 4 * (tid + NT_THREADS * i);
      if (c >= a.D) continue;
      const float xs[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
      const float gs[4] = {gm[i].x, gm[i].y, gm[i].z, gm[i].w}, bs[4] = {bt[i].x, bt[i].y, bt[i].z, bt[i].w};
      float o[4], ds4[4] = {1.f, 1.f, 1.f, 1.f};
      if (a.seed) mta_dropout_scale4(seed, (uint32_t)row, (uint32_t)c, a.drop_p, ds4);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = ((xs[j] - mu) * rs * gs[j] + bs[j]) * ds4[j];
      if (heads) {
        pa += (o[0] * wa4[i].x + o[1] * wa4[i].y) + (o[2] * wa4[i].z + o[3] * wa4[i].w);
        pb += (o[0] * wb4[i].x + o[1] * wb4[i].y) + (o[2] * wb4[i].z + o[3] * wb4[i].w);
      }
      if (a.y_f32) *reinterpret_cast<float4*>(a.y_f32 + (size_t)row * a.D + c) = make_float4(o[0], o[1], o[2], o[3]);
      if (a.y_bf16) {
        bf16x4 b;
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = (__bf16)o[j];
        *reinterpret_cast<bf16x4*>(a.y_bf16 + (size_t)row * a.D + c) = b;
      }
    }
    if (heads) {  // uniform: one more row reduction (fixed wave order)
      pa = wave_sum(pa);
      pb = wave_sum(pb);
      if (lane == 0) {
        redh[par][0][wave] = pa;
        redh[par][1][wave] = pb;
      }
      __syncthreads();
      if (tid == 0)
        a.ab[row] = make_float2(((redh[par][0][0] + redh[par][0][1]) + (redh[par][0][2] + redh[par][0][3])) + hba,
                                ((redh[par][1][0] + redh[par][1][1]) + (redh[par][1][2] + redh[par][1][3])) + hbb);
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) v[i] = vn[i];
  }
}

template <int VPT>
struct WideRow {
  float4 x[VPT], dy[VPT], dr[VPT];
  bf16x4 pre[VPT];
  float mu, rs;
};

template <int VPT>
__device__ __forceinline__ void wide_load(const NormArgs& a, int row, WideRow<VPT>& r) {
  const int tid = threadIdx.x;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = 4 * (tid + NT_THREADS * i);
    const bool ok = c < a.D;
    r.x[i] = ok ? ld4(a.x, a.xb, (size_t)row * a.ldx + c) : z;
    r.dy[i] = ok ? ld4(a.dy, a.dyb, (size_t)row * a.D + c) : z;
    r.dr[i] = (ok && a.dres) ? *reinterpret_cast<const float4*>(a.dres + (size_t)row * a.ldx + c) : z;
    if (ok && a.pre) r.pre[i] = *reinterpret_cast<const bf16x4*>(a.pre + (size_t)row * a.D + c);
  }
  r.mu = a.rms ? 0.f : a.mean[row];
  r.rs = a.rstd[row];
}

template <int VPT>
__global__ __launch_bounds__(NT_THREADS) void norm_bwd_wide_kernel(NormArgs a, int rows_per_block) {
  __shared__ float red[2][2][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float invD = 1.0f / (float)a.D;
  const uint64_t seed = a.seed ? *a.seed : 0ull;
  float4 gm[VPT];
  float dg[VPT][4], db[VPT][4];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = 4 * (tid + NT_THREADS * i);
    gm[i] = (c < a.D && a.gamma) ? *reinterpret_cast<const float4*>(a.gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
#pragma unroll
    for (int j = 0; j < 4; ++j) dg[i][j] = db[i][j] = 0.f;
  }
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(a.M, r0 + rows_per_block);
  if (r0 >= r1) return;
  // three row buffers in a fully unrolled ring (static register names: no buffer copy, which made every row wait
  // for the next row's loads), rows k + 1 and k + 2 in flight while row k is reduced; loads past the range re-read
  // the last row (unconditional: the compiler's vmcnt accounting stays exact)
  WideRow<VPT> rb[3];
  wide_load<VPT>(a, r0, rb[0]);
  wide_load<VPT>(a, min(r0 + 1, r1 - 1), rb[1]);
  for (int base = r0; base < r1; base += 3) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int row = base + k;
      if (row >= r1) break;
      wide_load<VPT>(a, min(row + 2, r1 - 1), rb[(k + 2) % 3]);
      WideRow<VPT>& cur = rb[k];
      float xh[VPT][4], g[VPT][4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int c = 4 * (tid + NT_THREADS * i);
        const bool ok = c < a.D;
        const float xs[4] = {cur.x[i].x, cur.x[i].y, cur.x[i].z, cur.x[i].w};
        const float ds[4] = {cur.dy[i].x, cur.dy[i].y, cur.dy[i].z, cur.dy[i].w};
        const float gs[4] = {gm[i].x, gm[i].y, gm[i].z, gm[i].w};
        float ds4[4] = {1.f, 1.f, 1.f, 1.f};
        if (a.seed && ok) mta_dropout_scale4(seed, (uint32_t)row, (uint32_t)c, a.drop_p, ds4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float d = ds[j] * ds4[j];
          xh[i][j] = ok ? (xs[j] - cur.mu) * cur.rs : 0.f;
          db[i][j] += d;
          dg[i][j] += d * xh[i][j];
          g[i][j] = d * gs[j];
          s1 += g[i][j];
          s2 += g[i][j] * xh[i][j];
        }
      }
      s1 = wave_sum(s1);
      s2 = wave_sum(s2);
      const int par = row & 1;
      if (lane == 0) {
        red[par][0][wave] = s1;
        red[par][1][wave] = s2;
      }
      __syncthreads();
      s1 = a.rms ? 0.f : ((red[par][0][0] + red[par][0][1]) + (red[par][0][2] + red[par][0][3])) * invD;
      s2 = ((red[par][1][0] + red[par][1][1]) + (red[par][1][2] + red[par][1][3])) * invD;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int c = 4 * (tid + NT_THREADS * i);
        if (c >= a.D) continue;
        const float rv[4] = {cur.dr[i].x, cur.dr[i].y, cur.dr[i].z, cur.dr[i].w};
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = cur.rs * (g[i][j] - s1 - xh[i][j] * s2) + rv[j];
          if (a.pre) o[j] *= mta_gelu_grad((float)cur.pre[i][j]);
        }
        if (a.dx_f32) *reinterpret_cast<float4*>(a.dx_f32 + (size_t)row * a.ldx + c) = make_float4(o[0], o[1], o[2], o[3]);
        if (a.dx_bf16) {
          bf16x4 b;
#pragma unroll
          for (int j = 0; j < 4; ++j) b[j] = (__bf16)o[j];
          *reinterpret_cast<bf16x4*>(a.dx_bf16 + (size_t)row * a.ldx + c) = b;
        }
      }
    }
  }
  if (!a.dgamma && !a.dbeta) return;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = 4 * (tid + NT_THREADS * i);
    if (c >= a.D) continue;
    if (a.dgamma)
      *reinterpret_cast<float4*>(a.part + (long)blockIdx.x * a.part_ld + c) = make_float4(dg[i][0], dg[i][1], dg[i][2], dg[i][3]);
    if (a.dbeta)
      *reinterpret_cast<float4*>(a.part + a.part_pass + (long)blockIdx.x * a.part_ld + c) =
          make_float4(db[i][0], db[i][1], db[i][2], db[i][3]);
  }
}

constexpr int NORM_BWD_MAX_BLOCKS = 1024;    // partial-row capacity of the static workspaces below
// The MLP's wide backward (pre != null, no residual gradient, x / dy both f32 or both bf16, D a multiple of
// 4 x 256 x VPT): every load unconditional and unconverted until use, so hipcc's vmcnt accounting keeps rows k + 1
// and k + 2 in flight while row k is reduced.  The generic kernel above branches per load (optional operands,
// bf16 -> f32 conversion in the loading branch): its waits drained the whole prefetch every row (r3 ISA).
template <int VPT, bool B16>
struct FastRow {
  typename std::conditional<B16, bf16x4, float4>::type x[VPT], dy[VPT];
  bf16x4 pre[VPT];
  float mu, rs;
  float2 dab;  // HD: d(alpha, beta) of the row
};

// GX: the row is gelu(pre) (NormArgs::gelu_x): no x load, x recomputed from the pre-activation the GELU' needs anyway
// HD: the row's dy is d_alpha wa + d_beta wb (fused heads): only d(alpha, beta) loaded
template <int VPT, bool B16, bool GX, bool HD>
__device__ __forceinline__ void fast_load(const NormArgs& a, const float* mean, int row, FastRow<VPT, B16>& r) {
  const int tid = threadIdx.x;
  if constexpr (HD) r.dab = a.ab[min(row, a.ab_rows - 1)];  // rows past ab_rows: zeroed at use
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = 4 * (tid + NT_THREADS * i);
    if constexpr (B16) {
      if constexpr (!GX) r.x[i] = *reinterpret_cast<const bf16x4*>(a.xb + (size_t)row * a.ldx + c);
      if constexpr (!HD) r.dy[i] = *reinterpret_cast<const bf16x4*>(a.dyb + (size_t)row * a.D + c);
    } else {
      if constexpr (!GX) r.x[i] = *reinterpret_cast<const float4*>(a.x + (size_t)row * a.ldx + c);
      if constexpr (!HD) r.dy[i] = *reinterpret_cast<const float4*>(a.dy + (size_t)row * a.D + c);
    }
    r.pre[i] = *reinterpret_cast<const bf16x4*>(a.pre + (size_t)row * a.D + c);
  }
  r.mu = mean[row];  // rstd when RMSNorm (selected at use)
  r.rs = a.rstd[row];
}

template <bool B16>
__device__ __forceinline__ void fast_f4(const typename std::conditional<B16, bf16x4, float4>::type& v, float (&o)[4]) {
  if constexpr (B16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (float)v[j];
  } else {
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
}

template <int VPT, bool B16, bool GX, bool HD>
__global__ __launch_bounds__(NT_THREADS) void norm_bwd_wide_fast_kernel(NormArgs a, int rows_per_block) {
  __shared__ float red[2][2][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float invD = 1.0f / (float)a.D;
  const uint64_t seed = a.seed ? *a.seed : 0ull;
  const float* mean = a.rms ? a.rstd : a.mean;
  float4 gm[VPT], bt[VPT], wa4[VPT], wb4[VPT];
  float dg[VPT][4], db[VPT][4], gwa[VPT][4], gwb[VPT][4];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = 4 * (tid + NT_THREADS * i);
    gm[i] = a.gamma ? *reinterpret_cast<const float4*>(a.gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    if constexpr (HD) {
      bt[i] = a.beta ? *reinterpret_cast<const float4*>(a.beta + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      wa4[i] = make_float4(a.hw_a[c], a.hw_a[c + 1], a.hw_a[c + 2], a.hw_a[c + 3]);
      wb4[i] = make_float4(a.hw_b[c], a.hw_b[c + 1], a.hw_b[c + 2], a.hw_b[c + 3]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) dg[i][j] = db[i][j] = gwa[i][j] = gwb[i][j] = 0.f;
  }
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(a.M, r0 + rows_per_block);
  if (r0 >= r1) return;
  FastRow<VPT, B16> rb[3];
  fast_load<VPT, B16, GX, HD>(a, mean, r0, rb[0]);
  fast_load<VPT, B16, GX, HD>(a, mean, min(r0 + 1, r1 - 1), rb[1]);
  for (int base = r0; base < r1; base += 3) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int row = base + k;
      if (row >= r1) break;
      fast_load<VPT, B16, GX, HD>(a, mean, min(row + 2, r1 - 1), rb[(k + 2) % 3]);
      const FastRow<VPT, B16>& cur = rb[k];
      const float mu = a.rms ? 0.f : cur.mu;
      float xh[VPT][4], g[VPT][4], gd[VPT][4];  // gd: GELU' (GX: computed with the GELU itself)
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int c = 4 * (tid + NT_THREADS * i);
        float xs[4], ds[4];
        if constexpr (GX) {
#pragma unroll
          for (int j = 0; j < 4; ++j) mta_gelu_and_grad((float)cur.pre[i][j], xs[j], gd[i][j]);
        } else {
          fast_f4<B16>(cur.x[i], xs);
        }
        float2 dab = make_float2(0.f, 0.f);
        if constexpr (HD) {
          dab = row < a.ab_rows ? cur.dab : make_float2(0.f, 0.f);
          ds[0] = dab.x * wa4[i].x + dab.y * wb4[i].x;
          ds[1] = dab.x * wa4[i].y + dab.y * wb4[i].y;
          ds[2] = dab.x * wa4[i].z + dab.y * wb4[i].z;
          ds[3] = dab.x * wa4[i].w + dab.y * wb4[i].w;
        } else {
          fast_f4<B16>(cur.dy[i], ds);
        }
        const float gs[4] = {gm[i].x, gm[i].y, gm[i].z, gm[i].w};
        float ds4[4] = {1.f, 1.f, 1.f, 1.f};
        if (a.seed) mta_dropout_scale4(seed, (uint32_t)row, (uint32_t)c, a.drop_p, ds4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float d = ds[j] * ds4[j];
          xh[i][j] = (xs[j] - mu) * cur.rs;
          if constexpr (HD) {  // the head input h = (xhat gamma + beta) * dropout scale
            const float bs4[4] = {bt[i].x, bt[i].y, bt[i].z, bt[i].w};
            const float hv = fmaf(xh[i][j], gs[j], bs4[j]) * ds4[j];
            gwa[i][j] = fmaf(dab.x, hv, gwa[i][j]);
            gwb[i][j] = fmaf(dab.y, hv, gwb[i][j]);
          }
          db[i][j] += d;
          dg[i][j] += d * xh[i][j];
          g[i][j] = d * gs[j];
          s1 += g[i][j];
          s2 += g[i][j] * xh[i][j];
        }
      }
      s1 = wave_sum(s1);
      s2 = wave_sum(s2);
      const int par = row & 1;
      if (lane == 0) {
        red[par][0][wave] = s1;
        red[par][1][wave] = s2;
      }
      __syncthreads();
      s1 = a.rms ? 0.f : ((red[par][0][0] + red[par][0][1]) + (red[par][0][2] + red[par][0][3])) * invD;
      s2 = ((red[par][1][0] + red[par][1][1]) + (red[par][1][2] + red[par][1][3])) * invD;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int c = 4 * (tid + NT_THREADS * i);
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = cur.rs * (g[i][j] - s1 - xh[i][j] * s2) * (GX ? gd[i][j] : mta_gelu_grad((float)cur.pre[i][j]));
        if (a.dx_f32) *reinterpret_cast<float4*>(a.dx_f32 + (size_t)row * a.ldx + c) = make_float4(o[0], o[1], o[2], o[3]);
        if (a.dx_bf16) {
          bf16x4 b;
#pragma unroll
          for (int j = 0; j < 4; ++j) b[j] = (__bf16)o[j];
          *reinterpret_cast<bf16x4*>(a.dx_bf16 + (size_t)row * a.ldx + c) = b;
        }
      }
    }
  }
  if constexpr (HD) {
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = 4 * (tid + NT_THREADS * i);
      *reinterpret_cast<float4*>(a.hpart + (long)blockIdx.x * a.part_ld + c) =
          make_float4(gwa[i][0], gwa[i][1], gwa[i][2], gwa[i][3]);
      *reinterpret_cast<float4*>(a.hpart + a.part_pass + (long)blockIdx.x * a.part_ld + c) =
          make_float4(gwb[i][0], gwb[i][1], gwb[i][2], gwb[i][3]);
    }
  }
  if (!a.dgamma && !a.dbeta) return;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = 4 * (tid + NT_THREADS * i);
    if (a.dgamma)
      *reinterpret_cast<float4*>(a.part + (long)blockIdx.x * a.part_ld + c) = make_float4(dg[i][0], dg[i][1], dg[i][2], dg[i][3]);
    if (a.dbeta)
      *reinterpret_cast<float4*>(a.part + a.part_pass + (long)blockIdx.x * a.part_ld + c) =
          make_float4(db[i][0], db[i][1], db[i][2], db[i][3]);
  }
}

// the wide backward: ~2 workgroups per CU, each a contiguous row range with two rows in flight (fewer, longer
// blocks: half the dgamma / dbeta partial rows of the r3 grid of 1024)
constexpr int NORM_BWD_WIDE_BLOCKS = 512;
// the wide forward's grid: ~4 workgroups per CU, each striding over rows with the next row in flight
constexpr int NORM_FWD_WIDE_BLOCKS = 1024;
// the one-wave-per-row backward's grid cap: transformer B=1 (M = 6,272 rows, D = 128) 0.714 ms at 512, 0.702 at
// 1024, 0.711 at 1,568 (one row per wave: the partial-row reduce grows) (profiles/r2_norm_bwd_cap_ab.txt)
constexpr int NORM_BWD_NARROW_BLOCKS = 1024;
// per-block column partials of dgamma / dbeta (static: no allocation, graph-capture safe; stream-ordered use)
__device__ float mta_norm_part[2][NORM_BWD_MAX_BLOCKS][2048];
__device__ float mta_norm_hpart[2][NORM_BWD_MAX_BLOCKS][2048];  // fused heads: head-weight gradient partial rows
// deferred reductions (D <= NORM_DEFER_D): each backward call gets its own slot and ONE batched launch sums every
// pending slot at the end of the encoder backward (9 launches -> 1 for the 4-layer transformer)
constexpr int NORM_DEFER_SLOTS = 12, NORM_DEFER_D = 256;
__device__ float mta_norm_part_slots[NORM_DEFER_SLOTS][2][NORM_BWD_MAX_BLOCKS][NORM_DEFER_D];

template <int VPL>
__global__ __launch_bounds__(NT_THREADS) void norm_bwd_kernel(NormArgs a) {
  __shared__ float red[4][4 * 64 * VPL];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float invD = 1.0f / (float)a.D;
  float dg[VPL][4], db[VPL][4];
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) dg[i][j] = db[i][j] = 0.f;

  // gamma before the row loop; the residual gradient and the GELU input with the row's x / dy (one dependent
  // round trip per row instead of three)
  float4 gm[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = 4 * (lane + 64 * i);
    gm[i] = (c < a.D && a.gamma) ? *reinterpret_cast<const float4*>(a.gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
  }
  for (int row = blockIdx.x * 4 + wave; row < a.M; row += gridDim.x * 4) {
    const float* xr = a.x + (size_t)row * a.ldx;
    const float* dyr = a.dy + (size_t)row * a.D;
    const float mu = a.rms ? 0.f : a.mean[row];
    const float rs = a.rstd[row];
    float xh[VPL][4], g[VPL][4];
    float4 rv[VPL], pf[VPL];
    bf16x4 pv[VPL];
    float s1 = 0.f, s2 = 0.f;  // sum(g*gamma), sum(g*gamma*xhat)
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = 4 * (lane + 64 * i);
      float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), dv = xv;
      rv[i] = xv;
      if (c < a.D) {
        xv = *reinterpret_cast<const float4*>(xr + c);
        dv = *reinterpret_cast<const float4*>(dyr + c);
        if (a.dres) rv[i] = *reinterpret_cast<const float4*>(a.dres + (size_t)row * a.ldx + c);
        if (a.pre) pv[i] = *reinterpret_cast<const bf16x4*>(a.pre + (size_t)row * a.D + c);
        if (a.pre_f) pf[i] = *reinterpret_cast<const float4*>(a.pre_f + (size_t)row * a.D + c);
      }
      const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, ds[4] = {dv.x, dv.y, dv.z, dv.w};
      const float gs[4] = {gm[i].x, gm[i].y, gm[i].z, gm[i].w};
      float ds4[4] = {1.f, 1.f, 1.f, 1.f};
      if (a.seed && c < a.D) mta_dropout_scale4(*a.seed, (uint32_t)row, (uint32_t)c, a.drop_p, ds4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float d = ds[j] * ds4[j];
        xh[i][j] = (xs[j] - mu) * rs;
        db[i][j] += d;
        dg[i][j] += d * xh[i][j];
        const float gg = d * gs[j];
        g[i][j] = gg;
        s1 += gg;
        s2 += gg * xh[i][j];
      }
    }
    s1 = a.rms ? 0.f : wave_sum(s1) * invD;
    s2 = wave_sum(s2) * invD;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = 4 * (lane + 64 * i);
      if (c >= a.D) continue;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = rs * (g[i][j] - s1 - xh[i][j] * s2);
      o[0] += rv[i].x;
      o[1] += rv[i].y;
      o[2] += rv[i].z;
      o[3] += rv[i].w;
      if (a.pre) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] *= mta_gelu_grad((float)pv[i][j]);
      }
      if (a.pre_f) {
        o[0] *= mta_gelu_grad(pf[i].x);
        o[1] *= mta_gelu_grad(pf[i].y);
        o[2] *= mta_gelu_grad(pf[i].z);
        o[3] *= mta_gelu_grad(pf[i].w);
      }
      if (a.dx_f32) *reinterpret_cast<float4*>(a.dx_f32 + (size_t)row * a.ldx + c) = make_float4(o[0], o[1], o[2], o[3]);
      if (a.dx_bf16) {
        bf16x4 b;
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = (__bf16)o[j];
        *reinterpret_cast<bf16x4*>(a.dx_bf16 + (size_t)row * a.ldx + c) = b;
      }
    }
  }
  if (!a.dgamma && !a.dbeta) return;
  // workgroup reduction of the per-wave column partials into this block's row of the partial workspace;
  // norm_param_reduce_kernel then sums the rows in block order (no same-address atomics: 512 blocks adding
  // to the same D columns serialised at L2, ~22 us per call at D=128; and the result is bit-reproducible)
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    float* dst = pass == 0 ? a.dgamma : a.dbeta;
    if (!dst) continue;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < VPL; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wave][4 * (lane + 64 * i) + j] = pass == 0 ? dg[i][j] : db[i][j];
    __syncthreads();
    for (int c = threadIdx.x; c < a.D; c += NT_THREADS)
      a.part[pass * a.part_pass + (long)blockIdx.x * a.part_ld + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// dgamma / dbeta += sum over the backward blocks' partial rows: one wave per column, lane l sums blocks
// l, l+64, ... (independent loads in flight), then a fixed-order wave reduction (bit-reproducible)
__global__ void norm_param_reduce_kernel(float* __restrict__ dgamma, float* __restrict__ dbeta, int D, int blocks) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (c >= 2 * D) return;
  const int pass = c / D, col = c % D;
  float* dst = pass == 0 ? dgamma : dbeta;
  if (!dst) return;
  float s = 0.f;
  for (int b = lane; b < blocks; b += 64) s += mta_norm_part[pass][b][col];
  s = wave_sum_dpp(s);
  if (lane == 0) dst[col] += s;
}

// the same column sums for the wide backward's many partial rows: lane = column (coalesced 256-B rows), the
// workgroup's 16 waves take every 16th partial row (16 independent loads in flight per lane), then the 16 wave
// partials are added in wave order through LDS (fixed order: bit-reproducible)
__global__ __launch_bounds__(1024) void norm_param_reduce_wide_kernel(float* __restrict__ dgamma,
                                                                       float* __restrict__ dbeta, int D, int blocks) {
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;  // over [0, 2D)
  const int pass = c >= D ? 1 : 0, col = c - pass * D;
  float* dst = pass == 0 ? dgamma : dbeta;
  float s = 0.f;
  if (c < 2 * D && dst) {
#pragma unroll 16
    for (int b = wave; b < blocks; b += 16) s += mta_norm_part[pass][b][col];
  }
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && c < 2 * D && dst) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += part[w][lane];
    dst[col] += t;
  }
}

// Column sums of the wide backward's partial rows, 32 columns per block (2D / 32 = 128 blocks at D = 2048, see
// param_reduce_cols), wave sums by a fixed xor tree, block sum in wave order (deterministic).  The 64-column
// form (64 blocks, 4 B per lane) took 8.3 us per call at mlp_large; a two-level form with a last-arriver ticket
// 12.9 us (its agent-scope release writes back the XCD's dirty L2 behind the norm backward) (r3 traces).
// part: a [2][NORM_BWD_MAX_BLOCKS][2048] partial region (mta_norm_part, or mta_norm_hpart for the fused heads)
__device__ __forceinline__ void param_reduce_cols(float* __restrict__ dgamma, float* __restrict__ dbeta, int D,
                                                  int blocks, const float* __restrict__ part, long pass_stride,
                                                  int bx);
__global__ __launch_bounds__(1024) void norm_param_reduce_cols_kernel(float* __restrict__ dgamma,
                                                                      float* __restrict__ dbeta, int D, int blocks,
                                                                      const float* __restrict__ part) {
  param_reduce_cols(dgamma, dbeta, D, blocks, part, (long)NORM_BWD_MAX_BLOCKS * 2048, blockIdx.x);
}
// deferred wide reductions (the MLP backward's dgamma / dbeta and fused-head partials of every layer): one launch,
// blockIdx.y = job, the same fixed-order sums
constexpr int NORM_WIDE_SLOTS = 8, NORM_WIDE_SLOT_BLOCKS = 512;
struct WideJob {
  const float* part;
  float* dgamma;
  float* dbeta;
  int D, blocks;
};
struct WideBatch {
  WideJob job[NORM_WIDE_SLOTS];
};
__global__ __launch_bounds__(1024) void norm_param_reduce_cols_batch_kernel(WideBatch b) {
  const WideJob& j = b.job[blockIdx.y];
  if ((int)blockIdx.x >= 2 * j.D / 32) return;
  param_reduce_cols(j.dgamma, j.dbeta, j.D, j.blocks, j.part, (long)NORM_WIDE_SLOT_BLOCKS * 2048, blockIdx.x);
}
// 32 columns per 1,024-thread block: 8 lanes x float4 = one whole 128-B line of a partial row per 8 lanes (16-column
// blocks read half lines: the 5-layer MLP batch reduce ran at ~1.8 TB/s), rows strided over 8-lane groups, then a
// fixed-order xor tree and wave-order sum: bit-reproducible
__device__ __forceinline__ void param_reduce_cols(float* __restrict__ dgamma, float* __restrict__ dbeta, int D,
                                                  int blocks, const float* __restrict__ part, long pass_stride,
                                                  int bx) {
  __shared__ float4 red[16][8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = bx * 32 + 4 * (lane & 7);  // over [0, 2D); D % 32 == 0: a block never straddles the planes
  const int pass = c >= D ? 1 : 0, col = c - pass * D;
  float* dst = pass == 0 ? dgamma : dbeta;
  if (dst == nullptr) return;  // uniform over the block
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b = wave * 8 + (lane >> 3); b < blocks; b += 128) {
    const float4 v = *reinterpret_cast<const float4*>(part + pass * pass_stride + (size_t)b * 2048 + col);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
#pragma unroll
  for (int m = 8; m < 64; m <<= 1) {
    s.x += __shfl_xor(s.x, m, 64);
    s.y += __shfl_xor(s.y, m, 64);
    s.z += __shfl_xor(s.z, m, 64);
    s.w += __shfl_xor(s.w, m, 64);
  }
  if (lane < 8) red[wave][lane] = s;
  __syncthreads();
  if (threadIdx.x < 8) {
    float4 t = red[0][threadIdx.x];
    for (int w = 1; w < 16; ++w) {
      const float4 v = red[w][threadIdx.x];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    dst[col] += t.x;  // parameter-gradient views need not be 16-B aligned
    dst[col + 1] += t.y;
    dst[col + 2] += t.z;
    dst[col + 3] += t.w;
  }
}

struct ReduceJob {
  const float* part;
  float* dgamma;
  float* dbeta;
  int D, blocks, ld;
  long pass;
};
struct ReduceBatch {
  ReduceJob job[NORM_DEFER_SLOTS];
};

// the same fixed-order column sums as norm_param_reduce_kernel, for every pending job (blockIdx.y)
__global__ void norm_param_reduce_batch_kernel(ReduceBatch b) {
  const ReduceJob& j = b.job[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (c >= 2 * j.D) return;
  const int pass = c / j.D, col = c % j.D;
  float* dst = pass == 0 ? j.dgamma : j.dbeta;
  if (!dst) return;
  float s = 0.f;
  for (int r = lane; r < j.blocks; r += 64) s += j.part[pass * j.pass + (long)r * j.ld + col];
  s = wave_sum_dpp(s);
  if (lane == 0) dst[col] += s;
}

bool defer_next = false;

struct DeferState {
  int n = 0;
  ReduceBatch batch;
  hipStream_t st = nullptr;
} deferred;

int norm_blocks(int M, bool bwd) {
  const int rows_per_block = 4;
  int b = (M + rows_per_block - 1) / rows_per_block;
  // backward: cap the grid so each wave reduces several rows before the per-column atomics
  static_assert(NORM_BWD_NARROW_BLOCKS <= NORM_BWD_MAX_BLOCKS, "partials sized for the grid cap");
  const int cap = bwd ? NORM_BWD_NARROW_BLOCKS : 4096;
  return b > cap ? cap : (b < 1 ? 1 : b);
}

}  // namespace

extern "C" int mta_cast_pad(int n, const float* const* src, void* const* dst, const int* rows, const int* cols,
                            const int* rows_p, const int* cols_p, const int* ld_src, uint64_t* seeds, int nseeds,
                            hipStream_t st) {
  if (n < 1 || n > 16 || nseeds < 0 || nseeds > 256 || (nseeds && !seeds)) return 1;
  CastArgs a;
  a.n = n;
  a.seeds = seeds;
  a.nseeds = nseeds;
  long maxe = 0;
  for (int i = 0; i < n; ++i) {
    a.item[i] = CastItem{src[i], static_cast<__bf16*>(dst[i]), rows[i], cols[i], rows_p[i], cols_p[i], ld_src[i]};
    const long e = (long)rows_p[i] * cols_p[i] / ((cols_p[i] & 7) == 0 ? 8 : 1);
    maxe = e > maxe ? e : maxe;
  }
  int bx = (int)((maxe + 255) / 256);
  bx = bx > 2048 ? 2048 : (bx < 1 ? 1 : bx);
  cast_pad_kernel<<<dim3(bx, n), 256, 0, st>>>(a);
  return 0;
}

// launch every deferred parameter reduction (one launch)
__device__ float mta_norm_wide_slots[NORM_WIDE_SLOTS][2][NORM_WIDE_SLOT_BLOCKS][2048];
struct WideDeferState {
  int n = 0;
  WideBatch batch;
  hipStream_t st = nullptr;
} wide_deferred;

void norm_wide_flush() {
  if (wide_deferred.n == 0) return;
  int maxD = 0;
  for (int i = 0; i < wide_deferred.n; ++i) maxD = std::max(maxD, wide_deferred.batch.job[i].D);
  norm_param_reduce_cols_batch_kernel<<<dim3(2 * maxD / 32, wide_deferred.n), 1024, 0, wide_deferred.st>>>(
      wide_deferred.batch);
  wide_deferred.n = 0;
}

// a wide deferred slot's partial base (two planes of NORM_WIDE_SLOT_BLOCKS x 2048), its job queued
// make room for k more slots before queuing any of them (a fused-head backward takes two: its norm slot, then its
// head slot -- a flush between the two would launch the first slot's reduction before its kernel has written it)
void norm_wide_reserve(int k, hipStream_t st) {
  if (wide_deferred.n + k > NORM_WIDE_SLOTS || (wide_deferred.n && wide_deferred.st != st)) norm_wide_flush();
}

float* norm_wide_slot(float* dgamma, float* dbeta, int D, int blocks, hipStream_t st) {
  if (wide_deferred.n == NORM_WIDE_SLOTS || (wide_deferred.n && wide_deferred.st != st)) norm_wide_flush();
  static float* base = [] {
    float* p = nullptr;
    (void)hipGetSymbolAddress(reinterpret_cast<void**>(&p), HIP_SYMBOL(mta_norm_wide_slots));
    return p;
  }();
  float* part = base + (long)wide_deferred.n * 2 * NORM_WIDE_SLOT_BLOCKS * 2048;
  wide_deferred.batch.job[wide_deferred.n] = WideJob{part, dgamma, dbeta, D, blocks};
  wide_deferred.st = st;
  ++wide_deferred.n;
  return part;
}

// drop every queued reduction unlaunched (a backward that raised part-way: its slots may never have been written)
extern "C" void mta_norm_discard() {
  wide_deferred.n = 0;
  deferred.n = 0;
}

extern "C" void mta_norm_flush() {
  norm_wide_flush();
  if (deferred.n == 0) return;
  int maxD = 0;
  for (int i = 0; i < deferred.n; ++i) maxD = deferred.batch.job[i].D > maxD ? deferred.batch.job[i].D : maxD;
  norm_param_reduce_batch_kernel<<<dim3((2 * maxD + 3) / 4, deferred.n), 256, 0, deferred.st>>>(deferred.batch);
  deferred.n = 0;
}

// A deferred dgamma / dbeta reduction slot for a kernel outside this file (the transformer's fused attention-half
// backward, csrc/tr_attn.hip): queues the job for mta_norm_flush (the same block-ordered, bit-reproducible sums) and
// returns the base of its partial rows: row b of pass p at base + p * (*pass) + b * (*ld).  Null when D or blocks
// exceed the slots.
extern "C" float* mta_norm_defer_slot(float* dgamma, float* dbeta, int D, int blocks, hipStream_t st, int* ld,
                                      long* pass) {
  if (D > NORM_DEFER_D || blocks < 1 || blocks > NORM_BWD_MAX_BLOCKS) return nullptr;
  if (deferred.n == NORM_DEFER_SLOTS || (deferred.n && deferred.st != st)) mta_norm_flush();
  static float* base = [] {
    float* p = nullptr;
    (void)hipGetSymbolAddress(reinterpret_cast<void**>(&p), HIP_SYMBOL(mta_norm_part_slots));
    return p;
  }();
  float* part = base + (long)deferred.n * 2 * NORM_BWD_MAX_BLOCKS * NORM_DEFER_D;
  *ld = NORM_DEFER_D;
  *pass = (long)NORM_BWD_MAX_BLOCKS * NORM_DEFER_D;
  deferred.batch.job[deferred.n] = ReduceJob{part, dgamma, dbeta, D, blocks, *ld, *pass};
  deferred.st = st;
  ++deferred.n;
  return part;
}

extern "C" int mta_norm(int bwd, const void* x, int x_bf16, int ldx, int M, int D, int rms, float eps,
                        const float* gamma, const float* beta, void* y_bf16, float* y_f32, float* mean, float* rstd,
                        const uint64_t* seed, float drop_p, const void* dy, int dy_bf16, const float* dres,
                        const void* pre, int pre_f32, void* dx_bf16, float* dx_f32, float* dgamma, float* dbeta,
                        const float* hw_a, const float* hb_a, const float* hw_b, const float* hb_b, float* ab,
                        int ab_rows, float* g_wa, float* g_wb, hipStream_t st) {
  if (D % 4 || ldx % 4 || D > 2048) return 1;
  // fp32 GELU input (32-true extras): the one-wave-per-row kernels (the wide ones stage pre as bf16)
  const bool wide_ok = D >= 1024 && !(pre && pre_f32);
  if ((x_bf16 || dy_bf16) && !wide_ok) return 2;  // bf16 row inputs: wide kernels only
  NormArgs a{};
  a.x = x_bf16 ? nullptr : static_cast<const float*>(x);
  a.xb = x_bf16 ? static_cast<const __bf16*>(x) : nullptr;
  a.gelu_x = x_bf16 == 2;  // 2: x is the bf16 GELU input (wide kernels)
  a.hw_a = hw_a;
  a.hw_b = hw_b;
  a.hb_a = hb_a;
  a.hb_b = hb_b;
  a.ab = reinterpret_cast<float2*>(ab);
  a.ab_rows = ab_rows;
  // fused heads: wide kernels only; the backward form is the GELU-on-load fast one, into both head gradients
  if (ab && !(wide_ok && hw_a && hw_b && (bwd ? (a.gelu_x && g_wa && g_wb && ab_rows > 0) : (hb_a && hb_b))))
    return 4;
  if (a.gelu_x && !(wide_ok && (!bwd || (pre && !pre_f32 && !dres && (D == 1024 || D == 2048))))) return 3;
  a.ldx = ldx;
  a.M = M;
  a.D = D;
  a.rms = rms;
  a.eps = eps;
  a.gamma = gamma;
  a.beta = beta;
  a.y_bf16 = static_cast<__bf16*>(y_bf16);
  a.y_f32 = y_f32;
  a.mean = mean;
  a.rstd = rstd;
  a.seed = seed;
  a.drop_p = drop_p;
  a.dy = dy_bf16 ? nullptr : static_cast<const float*>(dy);
  a.dyb = dy_bf16 ? static_cast<const __bf16*>(dy) : nullptr;
  a.dres = dres;
  a.pre = pre_f32 ? nullptr : static_cast<const __bf16*>(pre);
  a.pre_f = pre_f32 ? static_cast<const float*>(pre) : nullptr;
  a.dx_bf16 = static_cast<__bf16*>(dx_bf16);
  a.dx_f32 = dx_f32;
  a.dgamma = dgamma;
  a.dbeta = dbeta;
  const int vpl = (D + 255) / 256;
  const bool wide = wide_ok;
  int rows_per_block = 1;
  int blocks = norm_blocks(M, bwd != 0);
  if (wide && bwd) {
    // ~4 workgroups per CU, each a contiguous row range (partials: one row per block)
    rows_per_block = (M + NORM_BWD_WIDE_BLOCKS - 1) / NORM_BWD_WIDE_BLOCKS;
    if (rows_per_block < 2) rows_per_block = 2;
    blocks = (M + rows_per_block - 1) / rows_per_block;
  } else if (wide) {
    // the GELU-on-load form computes per element: twice the workgroups to hide its latency
    const int cap = a.gelu_x ? 2 * NORM_FWD_WIDE_BLOCKS : NORM_FWD_WIDE_BLOCKS;
    blocks = M < cap ? M : cap;
  }
  // deferred slot when the caller asked for it (dgamma pointer tagged by mta_norm_defer) and D fits
  const bool defer = bwd && (dgamma || dbeta) && defer_next && D <= NORM_DEFER_D;
  // wide backward of a deferring caller (the bf16 MLP): its dgamma / dbeta and fused-head partial rows go to wide
  // slots, reduced for every layer by ONE launch at mta_norm_flush (the per-call reduce was ~6 us + a launch gap)
  const bool defer_wide = bwd && defer_next && wide_ok && D % 32 == 0 && D <= 2048;
  defer_next = false;
  if (defer) {
    if (deferred.n == NORM_DEFER_SLOTS || (deferred.n && deferred.st != st)) mta_norm_flush();
    static float* base = [] {
      float* p = nullptr;
      (void)hipGetSymbolAddress(reinterpret_cast<void**>(&p), HIP_SYMBOL(mta_norm_part_slots));
      return p;
    }();
    a.part = base + (long)deferred.n * 2 * NORM_BWD_MAX_BLOCKS * NORM_DEFER_D;
    a.part_ld = NORM_DEFER_D;
    a.part_pass = (long)NORM_BWD_MAX_BLOCKS * NORM_DEFER_D;
    deferred.batch.job[deferred.n] = ReduceJob{a.part, dgamma, dbeta, D, blocks, a.part_ld, a.part_pass};
    deferred.st = st;
    ++deferred.n;
  } else {
    static float* base = [] {
      float* p = nullptr;
      (void)hipGetSymbolAddress(reinterpret_cast<void**>(&p), HIP_SYMBOL(mta_norm_part));
      return p;
    }();
    a.part = base;
    a.part_ld = 2048;
    a.part_pass = (long)NORM_BWD_MAX_BLOCKS * 2048;
  }
  const bool wide_slots = defer_wide && blocks <= NORM_WIDE_SLOT_BLOCKS;
  if (wide_slots) {
    a.part_pass = (long)NORM_WIDE_SLOT_BLOCKS * 2048;  // the plane stride of every wide slot (norm and head)
    norm_wide_reserve(bwd && a.ab ? 2 : 1, st);
    if (dgamma || dbeta) a.part = norm_wide_slot(dgamma, dbeta, D, blocks, st);
  }
#define NORM_LAUNCH(V)                                                          \
  if (bwd) norm_bwd_kernel<V><<<blocks, NT_THREADS, 0, st>>>(a);                \
  else norm_fwd_kernel<V><<<blocks, NT_THREADS, 0, st>>>(a);
  if (wide) {
    if (M > 0) {
      const bool b16 = a.gelu_x ? a.dyb != nullptr : a.xb != nullptr;
      const bool fast = a.pre && !a.dres && (a.gelu_x || b16 == (a.dyb != nullptr)) &&
                        (D == 1024 || D == 2048) && (a.rms || a.mean);
      if (bwd && a.ab && !fast) return 4;
      if (bwd && a.ab) {
        static float* hbase = [] {
          float* p = nullptr;
          (void)hipGetSymbolAddress(reinterpret_cast<void**>(&p), HIP_SYMBOL(mta_norm_hpart));
          return p;
        }();
        a.hpart = wide_slots ? norm_wide_slot(g_wa, g_wb, D, blocks, st) : hbase;
        // (the head slot shares the norm slot's plane stride: both NORM_WIDE_SLOT_BLOCKS x 2048 when deferred)
      }
#define NORM_FAST(V, B)                                                                                          \
  if (a.ab) norm_bwd_wide_fast_kernel<V, B, true, true><<<blocks, NT_THREADS, 0, st>>>(a, rows_per_block);       \
  else if (a.gelu_x) norm_bwd_wide_fast_kernel<V, B, true, false><<<blocks, NT_THREADS, 0, st>>>(a, rows_per_block); \
  else norm_bwd_wide_fast_kernel<V, B, false, false><<<blocks, NT_THREADS, 0, st>>>(a, rows_per_block);
      if (bwd && fast) {
        if (D == 1024) {
          if (b16) { NORM_FAST(1, true) } else { NORM_FAST(1, false) }
        } else {
          if (b16) { NORM_FAST(2, true) } else { NORM_FAST(2, false) }
        }
#undef NORM_FAST
      } else if (bwd) {
        if (D <= 1024) norm_bwd_wide_kernel<1><<<blocks, NT_THREADS, 0, st>>>(a, rows_per_block);
        else norm_bwd_wide_kernel<2><<<blocks, NT_THREADS, 0, st>>>(a, rows_per_block);
      } else {
        if (D <= 1024) {
          if (a.xb) norm_fwd_wide_kernel<1, true><<<blocks, NT_THREADS, 0, st>>>(a);
          else norm_fwd_wide_kernel<1, false><<<blocks, NT_THREADS, 0, st>>>(a);
        } else {
          if (a.xb) norm_fwd_wide_kernel<2, true><<<blocks, NT_THREADS, 0, st>>>(a);
          else norm_fwd_wide_kernel<2, false><<<blocks, NT_THREADS, 0, st>>>(a);
        }
      }
    }
  } else if (vpl <= 1) {
    NORM_LAUNCH(1)
  } else if (vpl <= 2) {
    NORM_LAUNCH(2)
  } else if (vpl <= 4) {
    NORM_LAUNCH(4)
  } else {
    NORM_LAUNCH(8)
  }
#undef NORM_LAUNCH
  if (bwd && (dgamma || dbeta) && wide && !wide_slots) {
    if (D % 32 == 0)
      norm_param_reduce_cols_kernel<<<2 * D / 32, 1024, 0, st>>>(dgamma, dbeta, D, blocks, a.part);
    else
      norm_param_reduce_wide_kernel<<<(2 * D + 63) / 64, 1024, 0, st>>>(dgamma, dbeta, D, blocks);
  } else if (bwd && (dgamma || dbeta) && !defer && !wide_slots)
    norm_param_reduce_kernel<<<(2 * D + 3) / 4, 256, 0, st>>>(dgamma, dbeta, D, blocks);
  if (bwd && a.ab && !wide_slots)  // the head weights' gradients (D in {1024, 2048}: the column-block reduction)
    norm_param_reduce_cols_kernel<<<2 * D / 32, 1024, 0, st>>>(g_wa, g_wb, D, blocks, a.hpart);
  return 0;
}

// sa += sum_i ab[i].x, sb += sum_i ab[i].y (the fused heads' bias gradients): one 1,024-thread workgroup, fixed
// order (thread-strided partials, then wave-order block sum): bit-reproducible
__global__ __launch_bounds__(1024) void pair_colsum_kernel(const float2* __restrict__ ab, int n, float* sa, float* sb) {
  __shared__ float part[2][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float x = 0.f, y = 0.f;
  for (int i = tid; i < n; i += 1024) {
    const float2 v = ab[i];
    x += v.x;
    y += v.y;
  }
  x = wave_sum(x);
  y = wave_sum(y);
  if (lane == 0) {
    part[0][wave] = x;
    part[1][wave] = y;
  }
  __syncthreads();
  if (tid < 2) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += part[tid][w];
    if (tid == 0) sa[0] += t;
    else sb[0] += t;
  }
}

extern "C" void mta_pair_colsum(const float* ab, int n, float* sa, float* sb, hipStream_t st) {
  pair_colsum_kernel<<<1, 1024, 0, st>>>(reinterpret_cast<const float2*>(ab), n, sa, sb);
}

// the next mta_norm backward call defers its parameter reduction to mta_norm_flush
extern "C" void mta_norm_defer() { defer_next = true; }
