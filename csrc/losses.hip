// Fused decoder losses: MSE decoder, Woodbury Gaussian NLL and MAE in one pass, with analytic
// gradients w.r.t. (alpha, beta) produced in the same pass.
//
// Reference semantics:
//   MSE : r_hat = alpha + beta * r_mkt ; mean((r_hat - r)^2) over all N*n   (src/model.py:192-206)
//   NLL : mu = alpha + beta * f_mean ; Sigma^-1 = Woodbury(beta, Psi^-1, f_var) built DENSE (K x K)
//         and 0.5 * (n (K ln 2pi - logdet Sigma^-1) + tr(D^T Sigma^-1 D))  (src/model.py:45-69,
//         src/common.py:50-78) -> here the O(K n) closed form of SURVEY.md A.1 (no K x K matrix, no LU).
//   MAE : mean |r_hat - r|                                                     (src/model.py:139)
// `windows` x `kwin` sequences: the reference's batch semantics (one Gaussian over all B*K
// sequences with window 0's factor) is windows=1, kwin=N, factor_stride=0; the
// corrected per-window batched NLL is windows=B, kwin=K, factor_stride=2.
#include "common.h"

namespace {

constexpr int TPB = 1024;
constexpr double LOG2PI = 1.8378770664093453;

__global__ __launch_bounds__(TPB) void decoder_losses_kernel(
    const float* __restrict__ ab,      // (N, 2): [alpha, beta]
    const float* __restrict__ y,       // (N, n, C): channel 0 = r_target, 1 = r_mkt
    const float* __restrict__ factor,  // (W', 2): [f_mean, f_var]
    const float* __restrict__ inv_psi, // (N)
    int N, int n, int C, int windows, int kwin, int factor_stride, int want_nll,
    float* __restrict__ out,           // [mse, nll, mae, sse]
    float* __restrict__ gmse,          // (N, 2) d mse / d (alpha, beta)
    float* __restrict__ gnll) {        // (N, 2) d nll / d (alpha, beta)
  extern __shared__ __attribute__((aligned(16))) float ut[];  // n floats
  __shared__ double red[TPB / 64][6];
  __shared__ double bcast[6];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float inv_cnt = 1.0f / ((float)N * (float)n);

  // Work split: one wave per sequence, lanes over the n target days (looping when n > 64);
  // every per-sequence sum is a wave reduction, u_t accumulates with LDS atomics whose
  // addresses are distinct within a wave instruction.
  const int nwaves = TPB / 64;
  // ---------------- MSE / MAE over all sequences -------------------------------------------
  double sse = 0.0, sae = 0.0;
  for (int i = wid; i < N; i += nwaves) {
    const float a = ab[2 * i], b = ab[2 * i + 1];
    const float* yi = y + (size_t)i * n * C;
    float se = 0.f, serm = 0.f, ss = 0.f, sa = 0.f;
    for (int t = lane; t < n; t += 64) {
      const float r = yi[t * C], rm = yi[t * C + 1];
      const float e = fmaf(b, rm, a) - r;
      se += e;
      serm = fmaf(e, rm, serm);
      ss = fmaf(e, e, ss);
      sa += fabsf(e);
    }
    se = wave_sum(se);
    serm = wave_sum(serm);
    sse += (double)wave_sum(ss);
    sae += (double)wave_sum(sa);
    if (lane == 0) {
      gmse[2 * i] = 2.f * se * inv_cnt;
      gmse[2 * i + 1] = 2.f * serm * inv_cnt;
    }
  }
  if (lane == 0) { red[wid][0] = sse; red[wid][1] = sae; }
  __syncthreads();
  if (tid == 0) {
    double s0 = 0, s1 = 0;
    for (int k = 0; k < nwaves; ++k) { s0 += red[k][0]; s1 += red[k][1]; }
    out[0] = (float)(s0 / ((double)N * n));
    out[2] = (float)(s1 / ((double)N * n));
    out[3] = (float)s0;
  }
  if (!want_nll) { if (tid == 0) out[1] = 0.f; return; }

  // ---------------- Woodbury NLL, window by window -------------------------------------------
  double nll_total = 0.0;
  for (int wdw = 0; wdw < windows; ++wdw) {
    const float fm = factor[wdw * factor_stride], fv = factor[wdw * factor_stride + 1];
    const int i0 = wdw * kwin;
    for (int t = tid; t < n; t += TPB) ut[t] = 0.f;
    __syncthreads();
    // pass 1: u_t = sum_i w_i b_i D_it ; partials of s = sum w b^2, sum log w, sum w D^2
    double s_wbb = 0.0, s_logw = 0.0, s_wdd = 0.0;
    for (int k = wid; k < kwin; k += nwaves) {
      const int i = i0 + k;
      const float a = ab[2 * i], b = ab[2 * i + 1], w = inv_psi[i];
      const float mu = fmaf(b, fm, a), wb = w * b;
      const float* yi = y + (size_t)i * n * C;
      float sdd = 0.f;
      for (int t = lane; t < n; t += 64) {
        const float D = yi[t * C] - mu;
        sdd = fmaf(D, D, sdd);
        atomicAdd(&ut[t], wb * D);
      }
      sdd = wave_sum(sdd);
      if (lane == 0) {
        s_wbb += (double)wb * b;
        s_logw += log((double)w);
        s_wdd += (double)w * sdd;
      }
    }
    __syncthreads();
    // U1 = sum_t u_t, U2 = sum_t u_t^2
    double s_u1 = 0.0, s_u2 = 0.0;
    for (int t = tid; t < n; t += TPB) { s_u1 += ut[t]; s_u2 += (double)ut[t] * ut[t]; }
    double v[5] = {s_wbb, s_logw, s_wdd, s_u1, s_u2};
#pragma unroll
    for (int m = 0; m < 5; ++m) v[m] = wave_sum_d(v[m]);
    if (lane == 0)
      for (int m = 0; m < 5; ++m) red[wid][m] = v[m];
    __syncthreads();
    if (tid == 0) {
      double acc[5] = {0, 0, 0, 0, 0};
      for (int k = 0; k < nwaves; ++k)
        for (int m = 0; m < 5; ++m) acc[m] += red[k][m];
      for (int m = 0; m < 5; ++m) bcast[m] = acc[m];
    }
    __syncthreads();
    const double den = 1.0 / (double)fv + bcast[0];
    const double logdet = bcast[1] - log((double)fv * den);
    const double U1 = bcast[3], U2 = bcast[4];
    const double quad = bcast[2] - U2 / den;
    nll_total += 0.5 * ((double)n * ((double)kwin * LOG2PI - logdet) + quad);
    // pass 2: gradients (derivation in masters_thesis_amd/ops/losses.py)
    const float fden = (float)den, fU1 = (float)U1, fU2 = (float)U2;
    for (int k = wid; k < kwin; k += nwaves) {
      const int i = i0 + k;
      const float a = ab[2 * i], b = ab[2 * i + 1], w = inv_psi[i];
      const float mu = fmaf(b, fm, a);
      const float* yi = y + (size_t)i * n * C;
      float sd = 0.f, ud = 0.f;
      for (int t = lane; t < n; t += 64) {
        const float D = yi[t * C] - mu;
        sd += D;
        ud = fmaf(ut[t], D, ud);
      }
      sd = wave_sum(sd);
      ud = wave_sum(ud);
      if (lane == 0) {
        const float wb = w * b;
        gnll[2 * i] = -w * sd + wb * fU1 / fden;
        gnll[2 * i + 1] = (float)n * wb / fden - fm * (w * sd - wb * fU1 / fden) - w * ud / fden +
                          fU2 * wb / (fden * fden);
      }
    }
    __syncthreads();
  }
  if (tid == 0) out[1] = (float)nll_total;
}

// d(alpha, beta) = g_mse * gmse + g_nll * gnll + g_mae * sign-term (MAE is eval-only: no grad)
__global__ void decoder_losses_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ gmse,
                                          const float* __restrict__ gnll, float* __restrict__ dab, int N2,
                                          int has_nll) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N2) return;
  float v = gout[0] * gmse[k];
  if (has_nll) v = fmaf(gout[1], gnll[k], v);
  dab[k] = v;
}

}  // namespace

extern "C" void mta_decoder_losses(const float* ab, const float* y, const float* factor, const float* inv_psi, int N,
                                   int n, int C, int windows, int kwin, int factor_stride, int want_nll, float* out,
                                   float* gmse, float* gnll, hipStream_t st) {
  decoder_losses_kernel<<<1, TPB, (size_t)((n + 3) & ~3) * sizeof(float), st>>>(
      ab, y, factor, inv_psi, N, n, C, windows, kwin, factor_stride, want_nll, out, gmse, gnll);
}

extern "C" void mta_decoder_losses_bwd(const float* gout, const float* gmse, const float* gnll, float* dab, int N,
                                       int has_nll, hipStream_t st) {
  const int N2 = 2 * N;
  decoder_losses_bwd_kernel<<<(N2 + 255) / 256, 256, 0, st>>>(gout, gmse, gnll, dab, N2, has_nll);
}
