// Fused decoder losses: alpha/beta heads, MSE decoder, Woodbury Gaussian NLL and MAE in one pass, with
// the analytic gradients w.r.t. (alpha, beta) produced in the same pass and the epoch metrics
// accumulated in place.
//
// Reference semantics:
//   heads: alpha = h_T w_a + b_a, beta = h_T w_b + b_b                          (src/model.py:96-97,105-108)
//   MSE : r_hat = alpha + beta * r_mkt ; mean((r_hat - r)^2) over all N*n         (src/model.py:192-206)
//   NLL : mu = alpha + beta * f_mean ; Sigma^-1 = Woodbury(beta, Psi^-1, f_var) built DENSE (K x K)
//         and 0.5 * (n (K ln 2pi - logdet Sigma^-1) + tr(D^T Sigma^-1 D))  (src/model.py:45-69,
//         src/common.py:50-78) -> here the O(K n) closed form of SURVEY.md A.1 (no K x K matrix, no LU).
//   MAE : mean |r_hat - r|                                                          (src/model.py:139)
//   total = c_nll * NLL + c_mse * MSE  (mse model: (0,1); nll: (1,0); combined: (1, mse_weight))
// `windows` x `kwin` sequences: the reference's batch semantics (one Gaussian over all B*K
// sequences with window 0's factor) is windows=1, kwin=N, factor_stride=0; the
// corrected per-window batched NLL is windows=B, kwin=K, factor_stride=2.
#include "common.h"

#ifndef MTA_STAMPS
#define MTA_STAMPS 0
#endif
#if MTA_STAMPS
// diagnostic build only (csrc/tools/losses_probe.hip): s_memtime at the phase boundaries of the training decoder
__device__ unsigned long long mta_loss_stamps[8];
#define LSTAMP(k)                                                                  \
  {                                                                                \
    __syncthreads();                                                               \
    if (threadIdx.x == 0) mta_loss_stamps[(k)] = __builtin_amdgcn_s_memtime();     \
  }
#else
#define LSTAMP(k)
#endif

namespace {

constexpr int TPB = 1024;
constexpr int NWAVES = TPB / 64;
// LDS floats of the u_t scratch: u_t itself plus one partial row per wave
__host__ __device__ inline size_t ut_floats(int n) { return (size_t)((n + 3) & ~3) + (size_t)NWAVES * n; }
constexpr double LOG2PI = 1.8378770664093453;

struct LossArgs {
  const float* y;        // (N, n, C): channel 0 = r_target, 1 = r_mkt
  const float* factor;   // (W', 2): [f_mean, f_var]
  const float* inv_psi;  // (N)
  int N, n, C, windows, kwin, factor_stride, want_nll;
  float c_nll, c_mse, batch_weight;
  float* out;            // [mse, nll, mae, total]
  float* gmse;           // (N, 2) d mse / d (alpha, beta)
  float* gnll;           // (N, 2) d nll / d (alpha, beta)
  double* acc;           // optional metric accumulator (8 doubles) or nullptr
  int dh_rows;           // training decoders: dh rows [N, dh_rows) are zero-filled (the encoder's padded rows)
};

// the encoder's padded rows of dh (their sequences do not exist): zeros, written by the decoder launch itself
__device__ __forceinline__ void zero_dh_pad(float* dh, int N, int H, int rows) {
  for (long i = (long)N * H + threadIdx.x; i < (long)rows * H; i += blockDim.x) dh[i] = 0.f;
}

// Work split: one wave per sequence, lanes over the n target days (looping when n > 64);
// every per-sequence sum is a wave reduction, u_t accumulates with LDS atomics whose
// addresses are distinct within a wave instruction.  `ab` may live in LDS or global memory.
// YL: the (r_target, r_mkt) pairs of every target day were staged in LDS as float2 (N, n) by the caller
// (one coalesced burst instead of a dependent global load per sequence iteration).
template <bool YL = false>
__device__ void losses_body(const float* ab, const LossArgs& A, float* ut, const float2* ys = nullptr) {
  __shared__ double red[NWAVES][6];
  __shared__ double bcast[6];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int N = A.N, n = A.n, C = A.C;
  const float inv_cnt = 1.0f / ((float)N * (float)n);

  // ---------------- MSE / MAE over all sequences -------------------------------------------
  double sse = 0.0, sae = 0.0;
  for (int i = wid; i < N; i += NWAVES) {
    const float a = ab[2 * i], b = ab[2 * i + 1];
    const float* yi = A.y + (size_t)i * n * C;
    float se = 0.f, serm = 0.f, ss = 0.f, sa = 0.f;
    for (int t = lane; t < n; t += 64) {
      const float r = YL ? ys[i * n + t].x : yi[t * C], rm = YL ? ys[i * n + t].y : yi[t * C + 1];
      const float e = fmaf(b, rm, a) - r;
      se += e;
      serm = fmaf(e, rm, serm);
      ss = fmaf(e, e, ss);
      sa += fabsf(e);
    }
    se = wave_sum_dpp(se);
    serm = wave_sum_dpp(serm);
    sse += (double)wave_sum_dpp(ss);
    sae += (double)wave_sum_dpp(sa);
    if (lane == 0) {
      A.gmse[2 * i] = 2.f * se * inv_cnt;
      A.gmse[2 * i + 1] = 2.f * serm * inv_cnt;
    }
  }
  if (lane == 0) { red[wid][0] = sse; red[wid][1] = sae; }
  __syncthreads();
  double s_sse = 0, s_sae = 0;
  for (int k = 0; k < NWAVES; ++k) { s_sse += red[k][0]; s_sae += red[k][1]; }
  const double mse = s_sse / ((double)N * n);

  // ---------------- Woodbury NLL, window by window -------------------------------------------
  double nll_total = 0.0;
  if (A.want_nll) {
    for (int wdw = 0; wdw < A.windows; ++wdw) {
      const float fm = A.factor[wdw * A.factor_stride], fv = A.factor[wdw * A.factor_stride + 1];
      const int i0 = wdw * A.kwin;
      // u_t partials per wave (row wid of ut + n), summed in wave order below: no float atomics, so the
      // loss and every gradient are bit-reproducible (deterministic mode relies on it)
      float* utw = ut + ((n + 3) & ~3);
      __syncthreads();
      for (int t = tid; t < NWAVES * n; t += TPB) utw[t] = 0.f;
      __syncthreads();
      // pass 1: u_t = sum_i w_i b_i D_it ; partials of s = sum w b^2, sum log w, sum w D^2
      double s_wbb = 0.0, s_logw = 0.0, s_wdd = 0.0;
      for (int k = wid; k < A.kwin; k += NWAVES) {
        const int i = i0 + k;
        const float a = ab[2 * i], b = ab[2 * i + 1], w = A.inv_psi[i];
        const float mu = fmaf(b, fm, a), wb = w * b;
        const float* yi = A.y + (size_t)i * n * C;
        float sdd = 0.f;
        for (int t = lane; t < n; t += 64) {
          const float D = (YL ? ys[i * n + t].x : yi[t * C]) - mu;
          sdd = fmaf(D, D, sdd);
          utw[wid * n + t] = fmaf(wb, D, utw[wid * n + t]);
        }
        sdd = wave_sum_dpp(sdd);
        if (lane == 0) {
          s_wbb += (double)wb * b;
          s_logw += (double)logf(w);  // fp32 log (fp64 log is a long software sequence), fp64 sum
          s_wdd += (double)w * sdd;
        }
      }
      __syncthreads();
      for (int t = tid; t < n; t += TPB) {
        float v = 0.f;
        for (int k = 0; k < NWAVES; ++k) v += utw[k * n + t];
        ut[t] = v;
      }
      __syncthreads();
      double s_u1 = 0.0, s_u2 = 0.0;
      for (int t = tid; t < n; t += TPB) { s_u1 += ut[t]; s_u2 += (double)ut[t] * ut[t]; }
      double v[5] = {s_wbb, s_logw, s_wdd, s_u1, s_u2};
#pragma unroll
      for (int m = 0; m < 5; ++m) v[m] = wave_sum_dpp(v[m]);
      if (lane == 0)
        for (int m = 0; m < 5; ++m) red[wid][m] = v[m];
      __syncthreads();
      if (tid == 0) {
        double acc[5] = {0, 0, 0, 0, 0};
        for (int k = 0; k < NWAVES; ++k)
          for (int m = 0; m < 5; ++m) acc[m] += red[k][m];
        for (int m = 0; m < 5; ++m) bcast[m] = acc[m];
      }
      __syncthreads();
      const double den = 1.0 / (double)fv + bcast[0];
      const double logdet = bcast[1] - log((double)fv * den);
      const double U1 = bcast[3], U2 = bcast[4];
      const double quad = bcast[2] - U2 / den;
      nll_total += 0.5 * ((double)n * ((double)A.kwin * LOG2PI - logdet) + quad);
      // pass 2: gradients (derivation in masters_thesis_amd/ops/losses.py)
      const float fden = (float)den, fU1 = (float)U1, fU2 = (float)U2;
      for (int k = wid; k < A.kwin; k += NWAVES) {
        const int i = i0 + k;
        const float a = ab[2 * i], b = ab[2 * i + 1], w = A.inv_psi[i];
        const float mu = fmaf(b, fm, a);
        const float* yi = A.y + (size_t)i * n * C;
        float sd = 0.f, ud = 0.f;
        for (int t = lane; t < n; t += 64) {
          const float D = (YL ? ys[i * n + t].x : yi[t * C]) - mu;
          sd += D;
          ud = fmaf(ut[t], D, ud);
        }
        sd = wave_sum_dpp(sd);
        ud = wave_sum_dpp(ud);
        if (lane == 0) {
          const float wb = w * b;
          A.gnll[2 * i] = -w * sd + wb * fU1 / fden;
          A.gnll[2 * i + 1] = (float)n * wb / fden - fm * (w * sd - wb * fU1 / fden) - w * ud / fden +
                              fU2 * wb / (fden * fden);
        }
      }
    }
  }
  if (tid == 0) {
    const double total = (double)A.c_nll * nll_total + (double)A.c_mse * mse;
    A.out[0] = (float)mse;
    A.out[1] = (float)nll_total;
    A.out[2] = (float)(s_sae / ((double)N * n));
    A.out[3] = (float)total;
    if (A.acc) {
      const double cnt = (double)N * n;
      A.acc[0] += s_sse;        // MSE: sum of squared errors
      A.acc[1] += cnt;          //      element count
      A.acc[2] += nll_total;    // NLL: loss sum
      A.acc[3] += 1.0;          //      update count (src/model.py:38-39)
      A.acc[4] += total * A.batch_weight;  // loss/total: batch-size weighted mean
      A.acc[5] += A.batch_weight;
      A.acc[6] += s_sae;        // MAE
      A.acc[7] += cnt;
    }
  }
}

__global__ __launch_bounds__(TPB) void decoder_losses_kernel(const float* __restrict__ ab, LossArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];  // ut_floats(n)
  losses_body(ab, A, smem);
}

// heads (two Linear(H,1)) computed in-kernel from h_T, then the losses
__global__ __launch_bounds__(TPB) void heads_losses_kernel(const float* __restrict__ h, int H,
                                                           const float* __restrict__ wa, const float* __restrict__ ba,
                                                           const float* __restrict__ wb, const float* __restrict__ bb,
                                                           float* __restrict__ ab_out, LossArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];  // 2N (ab) + n (u_t) floats
  float* ab = smem;
  float* ut = smem + 2 * ((A.N + 1) & ~1) + 4;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = wid; i < A.N; i += NWAVES) {
    float sa = 0.f, sb = 0.f;
    for (int k = lane; k < H; k += 64) {
      const float hv = h[(size_t)i * H + k];
      sa = fmaf(hv, wa[k], sa);
      sb = fmaf(hv, wb[k], sb);
    }
    sa = wave_sum_dpp(sa) + ba[0];
    sb = wave_sum_dpp(sb) + bb[0];
    if (lane == 0) {
      ab[2 * i] = sa;
      ab[2 * i + 1] = sb;
      ab_out[2 * i] = sa;
      ab_out[2 * i + 1] = sb;
    }
  }
  __syncthreads();
  losses_body(ab, A, ut);
}

// dh_T = d_a wa + d_b wb and the head weight / bias gradients (accumulated) from per-sequence d(alpha, beta)
// (`d`, 2N floats, LDS); single workgroup
__device__ void heads_bwd_body(const float* d, const float* __restrict__ h, int N, int H,
                               const float* __restrict__ wa, const float* __restrict__ wb, float* __restrict__ dh,
                               float* __restrict__ g_wa, float* __restrict__ g_ba, float* __restrict__ g_wb,
                               float* __restrict__ g_bb) {
  __shared__ float part[NWAVES][2][64 + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (dh) {
    for (int e = tid; e < N * H; e += TPB) {
      const int i = e / H, k = e % H;
      dh[e] = d[2 * i] * wa[k] + d[2 * i + 1] * wb[k];
    }
  }
  if (g_wa) {
    // wave w sums rows i = w, w+16, ... ; lane = column k (H <= 64 per pass)
    for (int k0 = 0; k0 < H; k0 += 64) {
      const int k = k0 + lane;
      float sa = 0.f, sb = 0.f, da = 0.f, db = 0.f;
      for (int i = wid; i < N; i += NWAVES) {
        const float hv = k < H ? h[(size_t)i * H + k] : 0.f;
        sa = fmaf(d[2 * i], hv, sa);
        sb = fmaf(d[2 * i + 1], hv, sb);
        da += d[2 * i];
        db += d[2 * i + 1];
      }
      part[wid][0][lane] = sa;
      part[wid][1][lane] = sb;
      if (lane == 0) { part[wid][0][64] = da; part[wid][1][64] = db; }
      __syncthreads();
      if (wid == 0) {
        float ta = 0.f, tb = 0.f;
        for (int w = 0; w < NWAVES; ++w) { ta += part[w][0][lane]; tb += part[w][1][lane]; }
        if (k < H) { g_wa[k] += ta; g_wb[k] += tb; }
        if (k0 == 0 && lane == 0) {
          float pa = 0.f, pb = 0.f;
          for (int w = 0; w < NWAVES; ++w) { pa += part[w][0][64]; pb += part[w][1][64]; }
          g_ba[0] += pa;
          g_bb[0] += pb;
        }
      }
      __syncthreads();
    }
  }
}

// Training step's whole decoder in ONE launch (the trainer's fused step: the loss is the step's root, so its
// upstream gradient is exactly 1): heads, every loss and metric, d(alpha, beta) = c_mse dMSE + c_nll dNLL,
// dh_T for the encoder's backward and the head weight gradients.  Replaces heads_losses + autograd's seed fill
// + heads_losses_bwd.  YL stages y in LDS (small N n).
template <bool YL>
__global__ __launch_bounds__(TPB) void heads_losses_train_kernel(
    const float* __restrict__ h, int H, const float* __restrict__ wa, const float* __restrict__ ba,
    const float* __restrict__ wb, const float* __restrict__ bb, LossArgs A, float* __restrict__ dh,
    float* __restrict__ g_wa, float* __restrict__ g_ba, float* __restrict__ g_wb, float* __restrict__ g_bb) {
  zero_dh_pad(dh, A.N, H, A.dh_rows);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int N = A.N, n = A.n;
  const int N2 = 2 * ((N + 1) & ~1);
  float* ab = smem;                      // 2N
  float* gm = ab + N2;                   // 2N  d mse / d(alpha, beta)
  float* gn = gm + N2;                   // 2N  d nll / d(alpha, beta)
  float* ut = gn + N2;                   // ut_floats(n)
  float2* ys = reinterpret_cast<float2*>(ut + ((ut_floats(n) + 3) & ~(size_t)3));  // (N, n) when YL
  float* hl = reinterpret_cast<float*>(ys + (size_t)N * n);                       // (N, H) when YL
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  LSTAMP(0)
  if constexpr (YL) {
    // one burst: every y pair and every h_T element in flight at once (the per-sequence loops below then
    // read LDS instead of paying a dependent global round trip per iteration)
    for (int e = tid; e < N * n; e += TPB) {
      const float* yp = A.y + (size_t)e * A.C;
      ys[e] = make_float2(yp[0], yp[1]);
    }
    for (int e = tid; e < N * H; e += TPB) hl[e] = h[e];
    __syncthreads();
    h = hl;
  }
  LSTAMP(1)
  for (int i = wid; i < N; i += NWAVES) {
    float sa = 0.f, sb = 0.f;
    for (int k = lane; k < H; k += 64) {
      const float hv = h[(size_t)i * H + k];
      sa = fmaf(hv, wa[k], sa);
      sb = fmaf(hv, wb[k], sb);
    }
    sa = wave_sum_dpp(sa) + ba[0];
    sb = wave_sum_dpp(sb) + bb[0];
    if (lane == 0) {
      ab[2 * i] = sa;
      ab[2 * i + 1] = sb;
    }
  }
  LSTAMP(2)
  __syncthreads();
  LossArgs L = A;
  L.gmse = gm;
  L.gnll = gn;
  losses_body<YL>(ab, L, ut, ys);
  LSTAMP(3)
  __syncthreads();
  const float cm = A.c_mse, cn = A.want_nll ? A.c_nll : 0.f;
  float* d = ab;  // alpha/beta are dead: reuse for d(alpha, beta)
  for (int k = tid; k < 2 * N; k += TPB) d[k] = cn != 0.f ? fmaf(cn, gn[k], cm * gm[k]) : cm * gm[k];
  __syncthreads();
  LSTAMP(4)
  heads_bwd_body(d, h, N, H, wa, wb, dh, g_wa, g_ba, g_wb, g_bb);
  LSTAMP(5)
}

// ---- register-resident training decoder (N <= 128, n <= 32, H in {16, 32, 64, 128}, <= 4 NLL windows) ----
// The wave-per-sequence kernel above loops 16 waves over the sequences with a full 64-lane reduction per
// sequence and quantity, and stages y and h_T through LDS first: 12.9 us for the headline step's MSE decoder
// (r2 rocprof), almost all of it dependent latency.  Here every input is loaded ONCE, straight into registers,
// in one burst (h_T as float4 rows, G = H/4 lanes per sequence; y as (r, r_mkt) pairs, one 32-lane half-wave
// per sequence, lane = target day), and every per-sequence quantity is a DPP half-wave (or G-lane) reduction
// whose result lands in every lane that needs it — the only LDS traffic is alpha/beta, the Woodbury u_t
// partials and d(alpha, beta).  Six block barriers in NLL mode, three in MSE mode.  All reductions run in a
// fixed order (bit-reproducible).
constexpr int RD_MAXP = 4, RD_MAXN = 128, RD_MAXW = 4;

// sum over aligned groups of G lanes (G in 4..32), the result in every lane of the group; whole waves only
template <int G, typename T>
__device__ __forceinline__ T group_sum(T v) {
  v += mta_dpp<0xB1>(v);  // quad_perm [1,0,3,2]
  v += mta_dpp<0x4E>(v);  // quad_perm [2,3,0,1]
  if constexpr (G >= 8) v += mta_dpp<0x141>(v);   // row_half_mirror: the other quad of the 8-lane half-row
  if constexpr (G >= 16) v += mta_dpp<0x140>(v);  // row_mirror: the other half-row
  if constexpr (G >= 32) v += __shfl_xor(v, 16);
  return v;
}

template <int G>
__global__ __launch_bounds__(TPB) void decoder_train_reg_kernel(
    const float* __restrict__ h, const float* __restrict__ wa, const float* __restrict__ ba,
    const float* __restrict__ wb, const float* __restrict__ bb, LossArgs A, float* __restrict__ dh,
    float* __restrict__ g_wa, float* __restrict__ g_ba, float* __restrict__ g_wb, float* __restrict__ g_bb) {
  constexpr int H = 4 * G, SPP = TPB / G;  // sequences per h pass
  zero_dh_pad(dh, A.N, H, A.dh_rows);
  __shared__ float2 ab[RD_MAXN], dab[RD_MAXN];
  __shared__ float cpart[RD_MAXN * 33];    // w_i b_i D_it, row i (stride 33); later the head-gradient partials
  __shared__ float upart[RD_MAXW][32][33];  // u_t partials: [window][sequence residue q][t]
  __shared__ float4 sq[RD_MAXN];            // per sequence: w b^2, log w, w sum_t D^2
  __shared__ float us[RD_MAXW][32];
  __shared__ double wsum[RD_MAXW][8];       // per window: s_wbb, s_logw, s_wdd, U1, U2, den, nll
  __shared__ double red[NWAVES][2];
  const int N = A.N, n = A.n, C = A.C;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int t = tid & 31, hw = tid >> 5;   // y mapping: half-wave hw owns sequence p*32 + hw, lane t = day t
  const int k4 = tid % G, hs = tid / G;    // h mapping: G lanes own sequence p*SPP + hs, float4 column k4
  const int yp = (N + 31) >> 5, hp = (N + SPP - 1) / SPP;
  const bool nll = A.want_nll != 0;
  // ---- one load burst: y pairs, inverse idiosyncratic variances, h_T rows, head weights ----
  float2 yv[RD_MAXP];
  float psi[RD_MAXP], fmv[RD_MAXP];
  float4 hv[RD_MAXP];
#pragma unroll
  for (int p = 0; p < RD_MAXP; ++p) {
    const int i = p * 32 + hw;
    yv[p] = make_float2(0.f, 0.f);
    psi[p] = 1.f;
    fmv[p] = 0.f;
    if (p < yp && i < N) {
      if (t < n) yv[p] = *reinterpret_cast<const float2*>(A.y + ((size_t)i * n + t) * C);
      if (nll) {
        psi[p] = A.inv_psi[i];
        fmv[p] = A.factor[(i / A.kwin) * A.factor_stride];
      }
    }
    const int ih = p * SPP + hs;
    hv[p] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p < hp && ih < N) hv[p] = *reinterpret_cast<const float4*>(h + (size_t)ih * H + 4 * k4);
  }
  // head weights are slices of the flat parameter buffer: scalar loads (no alignment to rely on)
  const float4 wa4 = make_float4(wa[4 * k4], wa[4 * k4 + 1], wa[4 * k4 + 2], wa[4 * k4 + 3]);
  const float4 wb4 = make_float4(wb[4 * k4], wb[4 * k4 + 1], wb[4 * k4 + 2], wb[4 * k4 + 3]);
  const float bav = ba[0], bbv = bb[0];
  // ---- heads: alpha_i = h_i . wa + ba, beta_i = h_i . wb + bb (G-lane reductions) ----
#pragma unroll
  for (int p = 0; p < RD_MAXP; ++p) {
    if (p < hp) {  // uniform
      const float4 x = hv[p];
      float sa = x.x * wa4.x + x.y * wa4.y + x.z * wa4.z + x.w * wa4.w;
      float sb = x.x * wb4.x + x.y * wb4.y + x.z * wb4.z + x.w * wb4.w;
      sa = group_sum<G>(sa);
      sb = group_sum<G>(sb);
      const int i = p * SPP + hs;
      if (k4 == 0 && i < N) ab[i] = make_float2(sa + bav, sb + bbv);
    }
  }
  __syncthreads();  // #1 alpha, beta
  // ---- MSE / MAE, NLL per-sequence terms (half-wave per sequence) ----
  const float inv_cnt = 1.0f / ((float)N * (float)n);
  float gma[RD_MAXP], gmb[RD_MAXP], sdv[RD_MAXP], dv[RD_MAXP];
  float ss = 0.f, sa = 0.f;
#pragma unroll
  for (int p = 0; p < RD_MAXP; ++p) {
    gma[p] = gmb[p] = sdv[p] = dv[p] = 0.f;
    if (p < yp) {  // uniform
      const int i = p * 32 + hw;
      const bool seq = i < N, valid = seq && t < n;
      const float2 abi = seq ? ab[i] : make_float2(0.f, 0.f);
      const float r = yv[p].x, rm = yv[p].y;
      const float e = valid ? fmaf(abi.y, rm, abi.x) - r : 0.f;
      ss = fmaf(e, e, ss);
      sa += fabsf(e);
      gma[p] = 2.f * group_sum<32>(e) * inv_cnt;
      gmb[p] = 2.f * group_sum<32>(e * rm) * inv_cnt;
      if (nll) {
        const float w = psi[p], mu = fmaf(abi.y, fmv[p], abi.x);
        const float D = valid ? r - mu : 0.f;
        dv[p] = D;
        const float sdd = group_sum<32>(D * D);
        sdv[p] = group_sum<32>(D);
        if (seq) {
          cpart[i * 33 + t] = w * abi.y * D;
          if (t == 0) sq[i] = make_float4(w * abi.y * abi.y, logf(w), w * sdd, 0.f);
        }
      }
    }
  }
  {
    const double s1 = wave_sum_dpp((double)ss), s2 = wave_sum_dpp((double)sa);
    if (lane == 0) {
      red[wid][0] = s1;
      red[wid][1] = s2;
    }
  }
  const float cm = A.c_mse, cn = nll ? A.c_nll : 0.f;
  if (nll) {
    const int W = A.windows, kwin = A.kwin;
    __syncthreads();  // #2 cpart, sq
    // ---- u_t partials (thread (q, t) sums the window's sequences i0 + q, i0 + q + 32, ...) and the
    //      per-window sequence sums (wave w) ----
    for (int w = 0; w < W; ++w) {
      float u = 0.f;
      for (int k = hw; k < kwin; k += 32) u += cpart[(w * kwin + k) * 33 + t];
      upart[w][hw][t] = u;
    }
    if (wid < W) {
      double s0 = 0.0, s1 = 0.0, s2 = 0.0;
      for (int k = lane; k < kwin; k += 64) {
        const float4 q = sq[wid * kwin + k];
        s0 += q.x;
        s1 += q.y;
        s2 += q.z;
      }
      s0 = wave_sum_dpp(s0);
      s1 = wave_sum_dpp(s1);
      s2 = wave_sum_dpp(s2);
      if (lane == 0) {
        wsum[wid][0] = s0;
        wsum[wid][1] = s1;
        wsum[wid][2] = s2;
      }
    }
    __syncthreads();  // #3 upart, window sums
    // ---- u_t, U1 = sum_t u_t, U2 = sum_t u_t^2 and the window's NLL (half-wave w) ----
    if (hw < W) {
      const int w = hw;
      float u = 0.f;
      for (int q = 0; q < 32; ++q) u += upart[w][q][t];
      u = t < n ? u : 0.f;
      us[w][t] = u;
      const double U1 = group_sum<32>((double)u), U2 = group_sum<32>((double)u * u);
      if (t == 0) {
        const float fv = A.factor[w * A.factor_stride + 1];
        const double den = 1.0 / (double)fv + wsum[w][0];
        const double logdet = wsum[w][1] - log((double)fv * den);
        wsum[w][3] = U1;
        wsum[w][4] = U2;
        wsum[w][5] = den;
        wsum[w][6] = 0.5 * ((double)n * ((double)kwin * LOG2PI - logdet) + (wsum[w][2] - U2 / den));
      }
    }
    __syncthreads();  // #4 u_t, U1, U2, den
    // ---- d(alpha, beta) with the NLL gradients (derivation in ops/losses.py) ----
#pragma unroll
    for (int p = 0; p < RD_MAXP; ++p) {
      if (p < yp) {
        const int i = p * 32 + hw;
        const int w = i < N ? i / kwin : 0;
        const float ud = group_sum<32>(us[w][t] * dv[p]);
        if (t == 0 && i < N) {
          const float b = ab[i].y, wi = psi[p], fm = fmv[p], sd = sdv[p];
          const float fden = (float)wsum[w][5], fU1 = (float)wsum[w][3], fU2 = (float)wsum[w][4];
          const float wbi = wi * b;
          const float gna = -wi * sd + wbi * fU1 / fden;
          const float gnb = (float)n * wbi / fden - fm * (wi * sd - wbi * fU1 / fden) - wi * ud / fden +
                            fU2 * wbi / (fden * fden);
          dab[i] = cn != 0.f ? make_float2(fmaf(cn, gna, cm * gma[p]), fmaf(cn, gnb, cm * gmb[p]))
                             : make_float2(cm * gma[p], cm * gmb[p]);
        }
      }
    }
  } else {
#pragma unroll
    for (int p = 0; p < RD_MAXP; ++p) {
      const int i = p * 32 + hw;
      if (p < yp && t == 0 && i < N) dab[i] = make_float2(cm * gma[p], cm * gmb[p]);
    }
  }
  __syncthreads();  // #5 d(alpha, beta)  (NLL) / #2 (MSE)
  // ---- dh_T = d_alpha wa + d_beta wb; head-weight gradients: column sums over the sequences ----
  float4 ga = make_float4(0.f, 0.f, 0.f, 0.f), gb = ga;
#pragma unroll
  for (int p = 0; p < RD_MAXP; ++p) {
    const int i = p * SPP + hs;
    if (p < hp && i < N) {
      const float2 d = dab[i];
      const float4 x = hv[p];
      *reinterpret_cast<float4*>(dh + (size_t)i * H + 4 * k4) =
          make_float4(d.x * wa4.x + d.y * wb4.x, d.x * wa4.y + d.y * wb4.y, d.x * wa4.z + d.y * wb4.z,
                      d.x * wa4.w + d.y * wb4.w);
      ga = make_float4(fmaf(d.x, x.x, ga.x), fmaf(d.x, x.y, ga.y), fmaf(d.x, x.z, ga.z), fmaf(d.x, x.w, ga.w));
      gb = make_float4(fmaf(d.y, x.x, gb.x), fmaf(d.y, x.y, gb.y), fmaf(d.y, x.z, gb.z), fmaf(d.y, x.w, gb.w));
    }
  }
#pragma unroll
  for (int m = G; m < 64; m <<= 1) {  // the wave's sequences sharing column k4
    ga.x += __shfl_xor(ga.x, m);
    ga.y += __shfl_xor(ga.y, m);
    ga.z += __shfl_xor(ga.z, m);
    ga.w += __shfl_xor(ga.w, m);
    gb.x += __shfl_xor(gb.x, m);
    gb.y += __shfl_xor(gb.y, m);
    gb.z += __shfl_xor(gb.z, m);
    gb.w += __shfl_xor(gb.w, m);
  }
  float4* gpart = reinterpret_cast<float4*>(cpart);  // cpart is dead after barrier #3 / never used (MSE)
  if (lane < G) {
    gpart[(wid * 2) * G + lane] = ga;
    gpart[(wid * 2 + 1) * G + lane] = gb;
  }
  __syncthreads();  // #6 head-gradient partials
  if (tid < 2 * G) {  // ordered sum over the waves
    const int which = tid / G, k = tid % G;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int w = 0; w < NWAVES; ++w) {
      const float4 v = gpart[(w * 2 + which) * G + k];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    float* g = (which ? g_wb : g_wa) + 4 * k;  // a slice of the flat gradient: no alignment to rely on
    g[0] += s.x;
    g[1] += s.y;
    g[2] += s.z;
    g[3] += s.w;
  } else if (wid == NWAVES - 1) {  // bias gradients: sum over the sequences
    float sa2 = 0.f, sb2 = 0.f;
    for (int i = lane; i < N; i += 64) {
      sa2 += dab[i].x;
      sb2 += dab[i].y;
    }
    sa2 = wave_sum_dpp(sa2);
    sb2 = wave_sum_dpp(sb2);
    if (lane == 0) {
      g_ba[0] += sa2;
      g_bb[0] += sb2;
    }
  } else if (tid == 2 * G) {  // losses + metric accumulators
    double s_sse = 0.0, s_sae = 0.0, nll_total = 0.0;
    for (int w = 0; w < NWAVES; ++w) {
      s_sse += red[w][0];
      s_sae += red[w][1];
    }
    if (nll)
      for (int w = 0; w < A.windows; ++w) nll_total += wsum[w][6];
    const double cnt = (double)N * n, mse = s_sse / cnt;
    const double total = (double)A.c_nll * nll_total + (double)A.c_mse * mse;
    A.out[0] = (float)mse;
    A.out[1] = (float)nll_total;
    A.out[2] = (float)(s_sae / cnt);
    A.out[3] = (float)total;
    if (A.acc) {
      A.acc[0] += s_sse;
      A.acc[1] += cnt;
      A.acc[2] += nll_total;
      A.acc[3] += 1.0;
      A.acc[4] += total * A.batch_weight;
      A.acc[5] += A.batch_weight;
      A.acc[6] += s_sae;
      A.acc[7] += cnt;
    }
  }
}

template <int G>
static void launch_decoder_reg(const float* h, const float* wa, const float* ba, const float* wb, const float* bb,
                               const LossArgs& A, float* dh, float* g_wa, float* g_ba, float* g_wb, float* g_bb,
                               hipStream_t st) {
  decoder_train_reg_kernel<G><<<1, TPB, 0, st>>>(h, wa, ba, wb, bb, A, dh, g_wa, g_ba, g_wb, g_bb);
}

static bool decoder_reg_fits(const float* h, const float* y, const float* dh, const float* wa, const float* wb,
                             int H, int N, int n, int C, int windows, int kwin, int want_nll) {
  const auto al = [](const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; };
  if (N < 1 || N > RD_MAXN || n < 1 || n > 32 || C < 2 || (C & 1)) return false;
  if (H != 16 && H != 32 && H != 64 && H != 128) return false;
  if ((N + 31) / 32 > RD_MAXP || ((long)N * H / 4 + TPB - 1) / TPB > RD_MAXP) return false;
  if (want_nll && (windows < 1 || windows > RD_MAXW || (long)windows * kwin != N)) return false;
  return al(h, 16) && al(dh, 16) && al(y, 8);
}

// backward: d(alpha, beta) from the saved per-sequence gradients, then dh_T and the head weight
// gradients (accumulated into the parameters' gradient views)
__global__ __launch_bounds__(TPB) void heads_losses_bwd_kernel(
    const float* __restrict__ g_mse, const float* __restrict__ g_nll, const float* __restrict__ g_total,  // nullable
    float c_nll, float c_mse, const float* __restrict__ gmse, const float* __restrict__ gnll, int has_nll,
    const float* __restrict__ h, int N, int H, const float* __restrict__ wa, const float* __restrict__ wb,
    float* __restrict__ dh, float* __restrict__ dab, float* __restrict__ g_wa, float* __restrict__ g_ba,
    float* __restrict__ g_wb, float* __restrict__ g_bb) {
  extern __shared__ __attribute__((aligned(16))) float d[];  // 2N
  const int tid = threadIdx.x;
  const float gt = g_total ? g_total[0] : 0.f;
  const float gm = (g_mse ? g_mse[0] : 0.f) + gt * c_mse;
  const float gn = has_nll ? (g_nll ? g_nll[0] : 0.f) + gt * c_nll : 0.f;
  for (int k = tid; k < 2 * N; k += TPB) {
    float v = gm * gmse[k];
    if (has_nll) v = fmaf(gn, gnll[k], v);
    d[k] = v;
    if (dab) dab[k] = v;
  }
  __syncthreads();
  heads_bwd_body(d, h, N, H, wa, wb, dh, g_wa, g_ba, g_wb, g_bb);
}

// ---- large N*H (wide encoders, big batches): grid-parallel heads and head backward ----
// heads: one wave per sequence, ab_out = [h.wa + ba, h.wb + bb]
__global__ __launch_bounds__(TPB) void heads_kernel(const float* __restrict__ h, int N, int H,
                                                    const float* __restrict__ wa, const float* __restrict__ ba,
                                                    const float* __restrict__ wb, const float* __restrict__ bb,
                                                    float* __restrict__ ab_out) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * NWAVES + (threadIdx.x >> 6);
  if (i >= N) return;
  float sa = 0.f, sb = 0.f;
  for (int k = 4 * lane; k < H; k += 256) {  // H % 4 == 0 on this path
    const float4 hv = *reinterpret_cast<const float4*>(h + (size_t)i * H + k);
    const float4 av = *reinterpret_cast<const float4*>(wa + k);
    const float4 bv = *reinterpret_cast<const float4*>(wb + k);
    sa += hv.x * av.x + hv.y * av.y + hv.z * av.z + hv.w * av.w;
    sb += hv.x * bv.x + hv.y * bv.y + hv.z * bv.z + hv.w * bv.w;
  }
  sa = wave_sum_dpp(sa);
  sb = wave_sum_dpp(sb);
  if (lane == 0) {
    ab_out[2 * i] = sa + ba[0];
    ab_out[2 * i + 1] = sb + bb[0];
  }
}

// d(alpha, beta) per sequence from the saved loss gradients
__global__ void heads_dab_kernel(const float* __restrict__ g_mse, const float* __restrict__ g_nll,
                                 const float* __restrict__ g_total, float c_nll, float c_mse,
                                 const float* __restrict__ gmse, const float* __restrict__ gnll, int has_nll, int N,
                                 float* __restrict__ dab) {
  const float gt = g_total ? g_total[0] : 0.f;
  const float gm = (g_mse ? g_mse[0] : 0.f) + gt * c_mse;
  const float gn = has_nll ? (g_nll ? g_nll[0] : 0.f) + gt * c_nll : 0.f;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < 2 * N; k += gridDim.x * blockDim.x) {
    float v = gm * gmse[k];
    if (has_nll) v = fmaf(gn, gnll[k], v);
    dab[k] = v;
  }
}

// dh = d_a wa + d_b wb (row-wise), head weight / bias gradients: per-block column partials over
// HB_ROWS rows, one atomic per column per block (contiguous, full-rate no-return atomics)
constexpr int HB_ROWS = 32;
__global__ __launch_bounds__(TPB) void heads_bwd_grid_kernel(const float* __restrict__ dab,
                                                             const float* __restrict__ h, int N, int H,
                                                             const float* __restrict__ wa,
                                                             const float* __restrict__ wb, float* __restrict__ dh,
                                                             float* __restrict__ g_wa, float* __restrict__ g_ba,
                                                             float* __restrict__ g_wb, float* __restrict__ g_bb,
                                                             float* __restrict__ part) {
  // part (deterministic mode): this block's column partials [wa H | wb H | ba | bb] with plain stores, summed in
  // block order by heads_part_reduce_kernel instead of the cross-block f32 atomics
  // grid (row blocks, column blocks of TPB): at N = 6,400, H = 2,048 the 200 row blocks alone left most CUs idle
  // (29 us per call); with the columns split too there are 1,600 workgroups and the same number of atomics
  float* my_part = part ? part + (size_t)blockIdx.x * (2 * H + 2) : nullptr;
  const int r0 = blockIdx.x * HB_ROWS;
  const int r1 = min(r0 + HB_ROWS, N);
  for (int k = blockIdx.y * TPB + threadIdx.x; k < H; k += gridDim.y * TPB) {
    const float a = wa[k], b = wb[k];
    float sa = 0.f, sb = 0.f;
    // the block's HB_ROWS h values of column k are loaded in one burst (a runtime-bounded row loop waited on each
    // row's load in turn: 35.6 us per call at N = 6,400, H = 2,048)
    float hv[HB_ROWS];
    if (g_wa) {
#pragma unroll
      for (int r = 0; r < HB_ROWS; ++r) hv[r] = r0 + r < r1 ? h[(size_t)(r0 + r) * H + k] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < HB_ROWS; ++r) {
      const int i = r0 + r;
      if (i >= r1) break;
      const float da = dab[2 * i], db = dab[2 * i + 1];
      if (dh) dh[(size_t)i * H + k] = da * a + db * b;
      if (g_wa) {
        sa = fmaf(da, hv[r], sa);
        sb = fmaf(db, hv[r], sb);
      }
    }
    if (g_wa) {
      if (my_part) {
        my_part[k] = sa;
        my_part[H + k] = sb;
      } else {
        atomicAdd(g_wa + k, sa);
        atomicAdd(g_wb + k, sb);
      }
    }
  }
  if (g_ba && blockIdx.y == 0 && threadIdx.x < 64) {
    float da = 0.f, db = 0.f;
    for (int i = r0 + threadIdx.x; i < r1; i += 64) {
      da += dab[2 * i];
      db += dab[2 * i + 1];
    }
    da = wave_sum_dpp(da);
    db = wave_sum_dpp(db);
    if (threadIdx.x == 0) {
      if (my_part) {
        my_part[2 * H] = da;
        my_part[2 * H + 1] = db;
      } else {
        atomicAdd(g_ba, da);
        atomicAdd(g_bb, db);
      }
    }
  }
}

// deterministic mode: column c of [g_wa | g_wb | g_ba | g_bb] += sum over blocks (in block order) of the partials
__global__ __launch_bounds__(256) void heads_part_reduce_kernel(const float* __restrict__ part, int nblocks, int H,
                                                               float* __restrict__ g_wa, float* __restrict__ g_ba,
                                                               float* __restrict__ g_wb, float* __restrict__ g_bb,
                                                               int has_w, int has_b) {
  const int c = blockIdx.x * 256 + threadIdx.x, W = 2 * H + 2;
  if (c >= W) return;
  float acc = 0.f;
  for (int b = 0; b < nblocks; ++b) acc += part[(size_t)b * W + c];
  if (c < H) {
    if (has_w) g_wa[c] += acc;
  } else if (c < 2 * H) {
    if (has_w) g_wb[c - H] += acc;
  } else if (has_b) {
    (c == 2 * H ? g_ba : g_bb)[0] += acc;
  }
}

int g_heads_deterministic = 0;

// small problems (the reference config: N = 100, H = 64) stay in the single fused workgroup
inline bool heads_big(int N, int H) { return (long)N * H > 32768 && H % 4 == 0; }

// ---- grid-parallel losses for large N (B = 64 windows = 6,400 sequences): ----
// decoder_losses_kernel is ONE workgroup whose 16 waves walk the sequences with a dependent y load per
// iteration, three passes: 316 us per call for mlp_large B=64 (r2 trace) - 11 % of that step.  Here:
//   L1 (windows x J blocks): per-sequence MSE gradient, block partials of sse / sae / sum w b^2 / sum log w /
//       sum w D^2 and of u_t (lane t owns day t: n <= 64) -> partial row P[w][j]
//   L2 (windows blocks): fixed-order sum of a window's J partial rows -> den, U1, U2, u_t, the window's NLL
//   L3 (sequence blocks): per-sequence NLL gradient; block 0 adds the window NLLs and the sse / sae partials
//       (fixed order) into the four loss scalars and the epoch metric accumulator
// Every sum has a fixed order (no float atomics): bit-reproducible like the single-workgroup kernel.
constexpr int LG_SEQ = 16;           // sequences per L1 block (4 per wave)
constexpr int LG_MAXJ = 256;         // partial rows per window
constexpr int LG_MAXP = 16384;       // partial rows in total
constexpr int LG_MAXW = 4096;        // windows
struct LgPart {
  double s[5];   // sse, sae, sum w b^2, sum log w, sum w D^2
  double pad[3];
  float ut[64];
};
struct LgWin {
  double nll;
  float den, u1, u2, pad;
  float ut[64];
};
__device__ LgPart mta_lg_part[LG_MAXP];
__device__ LgWin mta_lg_win[LG_MAXW];

// the grid losses from this many sequences on (the single-workgroup kernel took 36 us at N = 800, B = 8 windows)
constexpr int LG_MIN_N = 512;
inline bool losses_grid_ok(const LossArgs& A) {
  if (getenv("MTA_LOSSES_SINGLE")) return false;
  const int J = A.kwin <= 0 ? 0 : min(LG_MAXJ, (A.kwin + LG_SEQ - 1) / LG_SEQ);
  return A.N >= LG_MIN_N && A.n <= 64 && A.n >= 1 && A.windows <= LG_MAXW && (long)A.windows * A.kwin == A.N &&
         (long)A.windows * J <= LG_MAXP;
}

__global__ __launch_bounds__(256) void losses_grid_part_kernel(const float* __restrict__ ab, LossArgs A, int J, int S) {
  __shared__ double red[4][5];
  __shared__ float utp[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wdw = blockIdx.y, j = blockIdx.x;
  const int n = A.n, C = A.C;
  const float inv_cnt = 1.0f / ((float)A.N * (float)n);
  const float fm = A.want_nll ? A.factor[wdw * A.factor_stride] : 0.f;
  const int k0 = j * S, k1 = min(A.kwin, k0 + S);
  double sse = 0.0, sae = 0.0, wbb = 0.0, logw = 0.0, wdd = 0.0;
  float ut = 0.f;
  const bool tl = lane < n;
  for (int k = k0 + wave; k < k1; k += 4) {
    const int i = wdw * A.kwin + k;
    const float a = ab[2 * i], b = ab[2 * i + 1];
    const float* yi = A.y + (size_t)i * n * C;
    const float r = tl ? yi[lane * C] : 0.f, rm = tl ? yi[lane * C + 1] : 0.f;
    const float e = tl ? fmaf(b, rm, a) - r : 0.f;
    const float se = wave_sum_dpp(e);
    const float serm = wave_sum_dpp(e * rm);
    const float ss = wave_sum_dpp(e * e);
    const float sa = wave_sum_dpp(fabsf(e));
    if (lane == 0) {
      A.gmse[2 * i] = 2.f * se * inv_cnt;
      A.gmse[2 * i + 1] = 2.f * serm * inv_cnt;
    }
    sse += (double)ss;
    sae += (double)sa;
    if (A.want_nll) {
      const float w = A.inv_psi[i];
      const float mu = fmaf(b, fm, a), wb = w * b;
      const float D = tl ? r - mu : 0.f;
      const float sdd = wave_sum_dpp(D * D);
      ut = fmaf(wb, D, ut);
      wbb += (double)wb * b;
      logw += (double)logf(w);
      wdd += (double)w * sdd;
    }
  }
  if (lane == 0) {
    red[wave][0] = sse;
    red[wave][1] = sae;
    red[wave][2] = wbb;
    red[wave][3] = logw;
    red[wave][4] = wdd;
  }
  utp[wave][lane] = ut;
  __syncthreads();
  LgPart* P = mta_lg_part + (long)wdw * J + j;
  if (wave == 0) {
    P->ut[lane] = (utp[0][lane] + utp[1][lane]) + (utp[2][lane] + utp[3][lane]);
    if (lane < 5) P->s[lane] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  }
}

__global__ __launch_bounds__(64) void losses_grid_window_kernel(LossArgs A, int J) {
  const int lane = threadIdx.x, wdw = blockIdx.x, n = A.n;
  const LgPart* P = mta_lg_part + (long)wdw * J;
  float ut = 0.f;
  for (int j = 0; j < J; ++j) ut += P[j].ut[lane];  // lane t = day t, rows in order
  double s[3] = {0.0, 0.0, 0.0};                   // wbb, logw, wdd: lane-strided rows, then a fixed-order tree
  for (int j = lane; j < J; j += 64)
    for (int m = 0; m < 3; ++m) s[m] += P[j].s[2 + m];
  for (int m = 0; m < 3; ++m) s[m] = wave_sum_dpp(s[m]);
  const float utl = lane < n ? ut : 0.f;
  const double u1 = wave_sum_dpp((double)utl), u2 = wave_sum_dpp((double)utl * utl);
  LgWin* W = mta_lg_win + wdw;
  W->ut[lane] = utl;
  if (lane == 0) {
    const double fv = A.factor[wdw * A.factor_stride + 1];
    const double den = 1.0 / fv + s[0];
    const double logdet = s[1] - log(fv * den);
    const double quad = s[2] - u2 / den;
    W->nll = 0.5 * ((double)n * ((double)A.kwin * LOG2PI - logdet) + quad);
    W->den = (float)den;
    W->u1 = (float)u1;
    W->u2 = (float)u2;
  }
}

__global__ __launch_bounds__(256) void losses_grid_grad_kernel(const float* __restrict__ ab, LossArgs A, int J,
                                                               int nparts) {
  __shared__ double red[4][3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = A.n, C = A.C;
  if (A.want_nll) {
    const int i = blockIdx.x * 4 + wave;
    if (i < A.N) {
      const int wdw = i / A.kwin;
      const LgWin* W = mta_lg_win + wdw;
      const float fm = A.factor[wdw * A.factor_stride];
      const float a = ab[2 * i], b = ab[2 * i + 1], w = A.inv_psi[i];
      const float mu = fmaf(b, fm, a);
      const bool tl = lane < n;
      const float D = tl ? A.y[(size_t)i * n * C + lane * C] - mu : 0.f;
      const float sd = wave_sum_dpp(D);
      const float ud = wave_sum_dpp(tl ? W->ut[lane] * D : 0.f);
      if (lane == 0) {
        const float fden = W->den, fU1 = W->u1, fU2 = W->u2, wb = w * b;
        A.gnll[2 * i] = -w * sd + wb * fU1 / fden;
        A.gnll[2 * i + 1] = (float)n * wb / fden - fm * (w * sd - wb * fU1 / fden) - w * ud / fden +
                            fU2 * wb / (fden * fden);
      }
    }
  }
  if (blockIdx.x != 0) return;
  // scalars: lane-strided partial rows / windows per wave, fixed-order wave and block sums
  double sse = 0.0, sae = 0.0, nll = 0.0;
  for (int p = threadIdx.x; p < nparts; p += 256) {
    sse += mta_lg_part[p].s[0];
    sae += mta_lg_part[p].s[1];
  }
  if (A.want_nll)
    for (int w = threadIdx.x; w < A.windows; w += 256) nll += mta_lg_win[w].nll;
  sse = wave_sum_dpp(sse);
  sae = wave_sum_dpp(sae);
  nll = wave_sum_dpp(nll);
  if (lane == 0) {
    red[wave][0] = sse;
    red[wave][1] = sae;
    red[wave][2] = nll;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double s_sse = (red[0][0] + red[1][0]) + (red[2][0] + red[3][0]);
    const double s_sae = (red[0][1] + red[1][1]) + (red[2][1] + red[3][1]);
    const double nll_total = A.want_nll ? (red[0][2] + red[1][2]) + (red[2][2] + red[3][2]) : 0.0;
    const double cnt = (double)A.N * n;
    const double mse = s_sse / cnt;
    const double total = (double)A.c_nll * nll_total + (double)A.c_mse * mse;
    A.out[0] = (float)mse;
    A.out[1] = (float)nll_total;
    A.out[2] = (float)(s_sae / cnt);
    A.out[3] = (float)total;
    if (A.acc) {
      A.acc[0] += s_sse;
      A.acc[1] += cnt;
      A.acc[2] += nll_total;
      A.acc[3] += 1.0;
      A.acc[4] += total * A.batch_weight;
      A.acc[5] += A.batch_weight;
      A.acc[6] += s_sae;
      A.acc[7] += cnt;
    }
  }
}

// the decoder losses of `ab` (global memory) on the grid path when it applies, else the single workgroup
void launch_decoder_losses(const float* ab, const LossArgs& A, hipStream_t st) {
  if (losses_grid_ok(A)) {
    const int J = min(LG_MAXJ, (A.kwin + LG_SEQ - 1) / LG_SEQ);
    const int S = (A.kwin + J - 1) / J;
    losses_grid_part_kernel<<<dim3(J, A.windows), 256, 0, st>>>(ab, A, J, S);
    if (A.want_nll) losses_grid_window_kernel<<<A.windows, 64, 0, st>>>(A, J);
    losses_grid_grad_kernel<<<(A.N + 3) / 4, 256, 0, st>>>(ab, A, J, A.windows * J);
    return;
  }
  decoder_losses_kernel<<<1, TPB, ut_floats(A.n) * sizeof(float), st>>>(ab, A);
}

}  // namespace

extern "C" void mta_decoder_losses(const float* ab, const float* y, const float* factor, const float* inv_psi, int N,
                                   int n, int C, int windows, int kwin, int factor_stride, int want_nll, float c_nll,
                                   float c_mse, float batch_weight, float* out, float* gmse, float* gnll, double* acc,
                                   hipStream_t st) {
  LossArgs A{y, factor, inv_psi, N, n, C, windows, kwin, factor_stride, want_nll, c_nll, c_mse, batch_weight,
             out, gmse, gnll, acc};
  launch_decoder_losses(ab, A, st);
}

extern "C" void mta_heads_losses(const float* h, int H, const float* wa, const float* ba, const float* wb,
                                 const float* bb, float* ab_out, const float* y, const float* factor,
                                 const float* inv_psi, int N, int n, int C, int windows, int kwin, int factor_stride,
                                 int want_nll, float c_nll, float c_mse, float batch_weight, float* out, float* gmse,
                                 float* gnll, double* acc, hipStream_t st) {
  LossArgs A{y, factor, inv_psi, N, n, C, windows, kwin, factor_stride, want_nll, c_nll, c_mse, batch_weight,
             out, gmse, gnll, acc};
  if (heads_big(N, H)) {
    heads_kernel<<<(N + NWAVES - 1) / NWAVES, TPB, 0, st>>>(h, N, H, wa, ba, wb, bb, ab_out);
    launch_decoder_losses(ab_out, A, st);
    return;
  }
  const size_t lds = ((size_t)(2 * ((N + 1) & ~1) + 4) + ut_floats(n)) * sizeof(float);
  heads_losses_kernel<<<1, TPB, lds, st>>>(h, H, wa, ba, wb, bb, ab_out, A);
}

// fused training decoder (see heads_losses_train_kernel); returns -1 when the problem is too large for one
// workgroup's LDS (the caller keeps the forward / backward pair then)
extern "C" int mta_heads_losses_train(const float* h, int H, const float* wa, const float* ba, const float* wb,
                                      const float* bb, const float* y, const float* factor, const float* inv_psi,
                                      int N, int n, int C, int windows, int kwin, int factor_stride, int want_nll,
                                      float c_nll, float c_mse, float batch_weight, float* out, double* acc, float* dh,
                                      float* g_wa, float* g_ba, float* g_wb, float* g_bb, int dh_rows,
                                      hipStream_t st) {
  LossArgs A{y, factor, inv_psi, N, n, C, windows, kwin, factor_stride, want_nll, c_nll, c_mse, batch_weight,
             out, nullptr, nullptr, acc, dh_rows < N ? N : dh_rows};
  if (decoder_reg_fits(h, y, dh, wa, wb, H, N, n, C, windows, kwin, want_nll)) {
    switch (H) {
      case 16: launch_decoder_reg<4>(h, wa, ba, wb, bb, A, dh, g_wa, g_ba, g_wb, g_bb, st); break;
      case 32: launch_decoder_reg<8>(h, wa, ba, wb, bb, A, dh, g_wa, g_ba, g_wb, g_bb, st); break;
      case 64: launch_decoder_reg<16>(h, wa, ba, wb, bb, A, dh, g_wa, g_ba, g_wb, g_bb, st); break;
      default: launch_decoder_reg<32>(h, wa, ba, wb, bb, A, dh, g_wa, g_ba, g_wb, g_bb, st); break;
    }
    return 0;
  }
  const size_t base = ((size_t)(3 * 2 * ((N + 1) & ~1)) + ((ut_floats(n) + 3) & ~(size_t)3)) * sizeof(float);
  const size_t ybytes = (size_t)N * n * sizeof(float2) + (size_t)N * H * sizeof(float);  // y pairs + h_T
  if (base + ybytes <= 96 * 1024) {
    heads_losses_train_kernel<true><<<1, TPB, base + ybytes, st>>>(h, H, wa, ba, wb, bb, A, dh, g_wa, g_ba, g_wb,
                                                                   g_bb);
    return 0;
  }
  if (base > 60 * 1024) return -1;
  heads_losses_train_kernel<false><<<1, TPB, base, st>>>(h, H, wa, ba, wb, bb, A, dh, g_wa, g_ba, g_wb, g_bb);
  return 0;
}

extern "C" void mta_set_heads_deterministic(int on) { g_heads_deterministic = on ? 1 : 0; }
// floats of the partials buffer the deterministic grid path needs (0: none)
extern "C" long mta_heads_part_floats(int N, int H) {
  return heads_big(N, H) && g_heads_deterministic ? (long)((N + HB_ROWS - 1) / HB_ROWS) * (2 * H + 2) : 0;
}

extern "C" void mta_heads_losses_bwd(const float* g_mse, const float* g_nll, const float* g_total, float c_nll, float c_mse, const float* gmse,
                                     const float* gnll, int has_nll, const float* h, int N, int H, const float* wa,
                                     const float* wb, float* dh, float* dab, float* g_wa, float* g_ba, float* g_wb,
                                     float* g_bb, float* part, hipStream_t st) {
  if (heads_big(N, H) && dab) {
    const int nb = (N + HB_ROWS - 1) / HB_ROWS;
    heads_dab_kernel<<<(2 * N + 255) / 256, 256, 0, st>>>(g_mse, g_nll, g_total, c_nll, c_mse, gmse, gnll, has_nll,
                                                          N, dab);
    const bool det = part && (g_wa || g_ba);
    heads_bwd_grid_kernel<<<dim3(nb, (H + TPB - 1) / TPB), TPB, 0, st>>>(dab, h, N, H, wa, wb, dh, g_wa, g_ba, g_wb,
                                                                       g_bb, det ? part : nullptr);
    if (det)
      heads_part_reduce_kernel<<<(2 * H + 2 + 255) / 256, 256, 0, st>>>(part, nb, H, g_wa, g_ba, g_wb, g_bb,
                                                                        g_wa ? 1 : 0, g_ba ? 1 : 0);
    return;
  }
  heads_losses_bwd_kernel<<<1, TPB, (size_t)(2 * N) * sizeof(float), st>>>(g_mse, g_nll, g_total, c_nll, c_mse, gmse, gnll, has_nll, h,
                                                                           N, H, wa, wb, dh, dab, g_wa, g_ba, g_wb,
                                                                           g_bb);
}
