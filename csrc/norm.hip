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

namespace {

constexpr int NT_THREADS = 256;

struct CastItem {
  const float* src;
  __bf16* dst;
  int rows, cols, rows_p, cols_p, ld_src;
};
struct CastArgs {
  CastItem item[16];
  int n;
};

__global__ void cast_pad_kernel(CastArgs a) {
  const CastItem it = a.item[blockIdx.y];
  const long total = (long)it.rows_p * it.cols_p;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int r = (int)(e / it.cols_p), c = (int)(e % it.cols_p);
    const float v = (r < it.rows && c < it.cols) ? it.src[(size_t)r * it.ld_src + c] : 0.f;
    it.dst[e] = (__bf16)v;
  }
}

struct NormArgs {
  const float* x;
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
  const float* dres;    // [M][ldx] residual-stream gradient added to dx (or null)
  const __bf16* pre;    // [M][D] GELU input: dx *= gelu'(pre) (or null)
  __bf16* dx_bf16;      // [M][D]
  float* dx_f32;        // [M][ldx]
  float* dgamma;
  float* dbeta;
  float* part;          // per-block partial rows of dgamma / dbeta: [2][blocks][part_ld]
  int part_ld;
  long part_pass;       // floats between the dgamma and dbeta planes
};

template <int VPL>
__global__ __launch_bounds__(NT_THREADS) void norm_fwd_kernel(NormArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float invD = 1.0f / (float)a.D;
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
      float o[4] = {(v[i].x - mu) * rs, (v[i].y - mu) * rs, (v[i].z - mu) * rs, (v[i].w - mu) * rs};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (a.gamma) o[j] *= a.gamma[c + j];
        if (a.beta) o[j] += a.beta[c + j];
        if (a.seed) o[j] *= mta_dropout_scale(*a.seed, (uint32_t)row, (uint32_t)(c + j), a.drop_p);
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

constexpr int NORM_BWD_MAX_BLOCKS = 512;
// per-block column partials of dgamma / dbeta (static: no allocation, graph-capture safe; stream-ordered use)
__device__ float mta_norm_part[2][NORM_BWD_MAX_BLOCKS][2048];
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

  for (int row = blockIdx.x * 4 + wave; row < a.M; row += gridDim.x * 4) {
    const float* xr = a.x + (size_t)row * a.ldx;
    const float* dyr = a.dy + (size_t)row * a.D;
    const float mu = a.rms ? 0.f : a.mean[row];
    const float rs = a.rstd[row];
    float xh[VPL][4], g[VPL][4];
    float s1 = 0.f, s2 = 0.f;  // sum(g*gamma), sum(g*gamma*xhat)
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = 4 * (lane + 64 * i);
      float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), dv = xv;
      if (c < a.D) {
        xv = *reinterpret_cast<const float4*>(xr + c);
        dv = *reinterpret_cast<const float4*>(dyr + c);
      }
      const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, ds[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float d = ds[j];
        if (a.seed && c < a.D) d *= mta_dropout_scale(*a.seed, (uint32_t)row, (uint32_t)(c + j), a.drop_p);
        xh[i][j] = (xs[j] - mu) * rs;
        db[i][j] += d;
        dg[i][j] += d * xh[i][j];
        const float gg = a.gamma && c < a.D ? d * a.gamma[c + j] : d;
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
      if (a.dres) {
        const float4 r = *reinterpret_cast<const float4*>(a.dres + (size_t)row * a.ldx + c);
        o[0] += r.x;
        o[1] += r.y;
        o[2] += r.z;
        o[3] += r.w;
      }
      if (a.pre) {
        const bf16x4 p = *reinterpret_cast<const bf16x4*>(a.pre + (size_t)row * a.D + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] *= mta_gelu_grad((float)p[j]);
      }
      if (a.dx_f32) *reinterpret_cast<float4*>(a.dx_f32 + (size_t)row * a.ldx + c) = make_float4(o[0], o[1], o[2], o[3]);
      if (a.dx_bf16) {
        bf16x4 b;
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = (__bf16)o[j];
        *reinterpret_cast<bf16x4*>(a.dx_bf16 + (size_t)row * a.D + c) = b;
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
  const int cap = bwd ? NORM_BWD_MAX_BLOCKS : 4096;
  return b > cap ? cap : (b < 1 ? 1 : b);
}

}  // namespace

extern "C" int mta_cast_pad(int n, const float* const* src, void* const* dst, const int* rows, const int* cols,
                            const int* rows_p, const int* cols_p, const int* ld_src, hipStream_t st) {
  if (n < 1 || n > 16) return 1;
  CastArgs a;
  a.n = n;
  long maxe = 0;
  for (int i = 0; i < n; ++i) {
    a.item[i] = CastItem{src[i], static_cast<__bf16*>(dst[i]), rows[i], cols[i], rows_p[i], cols_p[i], ld_src[i]};
    const long e = (long)rows_p[i] * cols_p[i];
    maxe = e > maxe ? e : maxe;
  }
  int bx = (int)((maxe + 255) / 256);
  bx = bx > 2048 ? 2048 : (bx < 1 ? 1 : bx);
  cast_pad_kernel<<<dim3(bx, n), 256, 0, st>>>(a);
  return 0;
}

// launch every deferred parameter reduction (one launch)
extern "C" void mta_norm_flush() {
  if (deferred.n == 0) return;
  int maxD = 0;
  for (int i = 0; i < deferred.n; ++i) maxD = deferred.batch.job[i].D > maxD ? deferred.batch.job[i].D : maxD;
  norm_param_reduce_batch_kernel<<<dim3((2 * maxD + 3) / 4, deferred.n), 256, 0, deferred.st>>>(deferred.batch);
  deferred.n = 0;
}

extern "C" int mta_norm(int bwd, const float* x, int ldx, int M, int D, int rms, float eps, const float* gamma,
                        const float* beta, void* y_bf16, float* y_f32, float* mean, float* rstd,
                        const uint64_t* seed, float drop_p, const float* dy, const float* dres, const void* pre,
                        void* dx_bf16, float* dx_f32, float* dgamma, float* dbeta, hipStream_t st) {
  if (D % 4 || ldx % 4 || D > 2048) return 1;
  NormArgs a;
  a.x = x;
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
  a.dy = dy;
  a.dres = dres;
  a.pre = static_cast<const __bf16*>(pre);
  a.dx_bf16 = static_cast<__bf16*>(dx_bf16);
  a.dx_f32 = dx_f32;
  a.dgamma = dgamma;
  a.dbeta = dbeta;
  const int vpl = (D + 255) / 256;
  const int blocks = norm_blocks(M, bwd != 0);
  // deferred slot when the caller asked for it (dgamma pointer tagged by mta_norm_defer) and D fits
  const bool defer = bwd && (dgamma || dbeta) && defer_next && D <= NORM_DEFER_D;
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
#define MTA_NORM_LAUNCH(V)                                                      \
  if (bwd) norm_bwd_kernel<V><<<blocks, NT_THREADS, 0, st>>>(a);                \
  else norm_fwd_kernel<V><<<blocks, NT_THREADS, 0, st>>>(a);
  if (vpl <= 1) {
    MTA_NORM_LAUNCH(1)
  } else if (vpl <= 2) {
    MTA_NORM_LAUNCH(2)
  } else if (vpl <= 4) {
    MTA_NORM_LAUNCH(4)
  } else {
    MTA_NORM_LAUNCH(8)
  }
#undef MTA_NORM_LAUNCH
  if (bwd && (dgamma || dbeta) && !defer)
    norm_param_reduce_kernel<<<(2 * D + 3) / 4, 256, 0, st>>>(dgamma, dbeta, D, blocks);
  return 0;
}

// the next mta_norm backward call defers its parameter reduction to mta_norm_flush
extern "C" void mta_norm_defer() { defer_next = true; }
