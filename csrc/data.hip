// Dataset-build kernels (run once per dataset, not in the train step):
//
//   mta_dgp            synthetic single-factor DGP (reference `src/data.py:49-59`):
//                      r[k][s] = alpha_k + beta_k * r_mkt[s] + eps[k][s],  r_mkt, eps ~ loc + scale * t_df,
//                      alpha, beta ~ Normal; counter-based (seed, stream, index) hashing -> Box-Muller normals;
//                      Student-t with integer df as z / sqrt(chi2_df / df), chi2_df = sum of df squared normals
//                      (exact for the configs' df = 5).  One launch for the market, one for the stocks.
//   mta_ols_features   OLS targets of the future window (reference `src/common.py:132-149`):
//                      per (window, stock) closed-form simple regression of the stock on the market with the
//                      reference's pinv semantics for a constant regressor, unbiased residual variance ->
//                      inv_psi, and per window the market's [mean, unbiased var].
#include "common.h"

namespace {

__device__ __forceinline__ float uniform_open(uint64_t seed, uint32_t stream, uint32_t idx) {
  // (0, 1]: Box-Muller needs log(u) finite
  return ((float)(mta_hash3(seed, stream, idx) >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float normal(uint64_t seed, uint32_t stream, uint32_t idx) {
  const float u1 = uniform_open(seed, stream, 2 * idx);
  const float u2 = uniform_open(seed, stream, 2 * idx + 1);
  return sqrtf(-2.0f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}

// Student-t(df) for integer df: z / sqrt(chi2_df / df)
__device__ __forceinline__ float student_t(uint64_t seed, uint32_t stream, uint32_t idx, int df) {
  const float z = normal(seed, stream, (uint32_t)(idx * (df + 1)));
  float chi = 0.f;
  for (int i = 1; i <= df; ++i) {
    const float g = normal(seed, stream, (uint32_t)(idx * (df + 1) + i));
    chi = fmaf(g, g, chi);
  }
  return z * rsqrtf(chi / (float)df);
}

struct DgpArgs {
  uint64_t seed;
  int n_stocks;
  long n_samples;
  int mkt_df, idio_df;
  float mkt_loc, mkt_scale, idio_loc, idio_scale, a_loc, a_scale, b_loc, b_scale;
  float* r_market;  // (n_samples)
  float* r_stocks;  // (n_stocks, n_samples)
  float* alphas;    // (n_stocks)
  float* betas;     // (n_stocks)
};

__global__ void dgp_market_kernel(DgpArgs a) {
  for (long s = blockIdx.x * (long)blockDim.x + threadIdx.x; s < a.n_samples; s += (long)gridDim.x * blockDim.x)
    a.r_market[s] = a.mkt_loc + a.mkt_scale * student_t(a.seed, 0x4D4B54u, (uint32_t)s, a.mkt_df);
  if (blockIdx.x == 0) {
    for (int k = threadIdx.x; k < a.n_stocks; k += blockDim.x) {
      a.alphas[k] = a.a_loc + a.a_scale * normal(a.seed, 0x414C50u, (uint32_t)k);
      a.betas[k] = a.b_loc + a.b_scale * normal(a.seed, 0x424554u, (uint32_t)k);
    }
  }
}

// stock k = blockIdx.y; fused alpha + beta * r_mkt + eps
__global__ void dgp_stocks_kernel(DgpArgs a) {
  const int k = blockIdx.y;
  const float al = a.alphas[k], be = a.betas[k];
  float* out = a.r_stocks + (size_t)k * a.n_samples;
  const uint32_t stream = 0x10000u + (uint32_t)k;
  for (long s = blockIdx.x * (long)blockDim.x + threadIdx.x; s < a.n_samples; s += (long)gridDim.x * blockDim.x) {
    const float eps = a.idio_loc + a.idio_scale * student_t(a.seed, stream, (uint32_t)s, a.idio_df);
    out[s] = fmaf(be, a.r_market[s], al + eps);
  }
}

// one thread per (window, stock); target (W, K, n, C): channel 0 = stock, 1 = market
__global__ void ols_features_kernel(const float* __restrict__ target, int W, int K, int n, int C,
                                    float* __restrict__ alphas, float* __restrict__ betas,
                                    float* __restrict__ factor, float* __restrict__ inv_psi) {
  const long id = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (id >= (long)W * K) return;
  const int wdx = (int)(id / K), k = (int)(id % K);
  const float* ys = target + ((size_t)wdx * K + k) * n * C;
  const float* xs = target + ((size_t)wdx * K) * n * C + 1;  // market from stock 0's rows (same for all k)
  float xm = 0.f, ym = 0.f;
  for (int i = 0; i < n; ++i) {
    xm += xs[(size_t)i * C];
    ym += ys[(size_t)i * C];
  }
  xm /= (float)n;
  ym /= (float)n;
  float sxx = 0.f, sxy = 0.f;
  for (int i = 0; i < n; ++i) {
    const float xc = xs[(size_t)i * C] - xm;
    sxx = fmaf(xc, xc, sxx);
    sxy = fmaf(xc, ys[(size_t)i * C], sxy);
  }
  float alpha, beta;
  if (sxx <= 0.f) {  // pinv semantics for a constant regressor: min-norm [a, b] with a + b x0 = mean(y)
    const float x0 = xs[0];
    beta = ym * x0 / (1.f + x0 * x0);
    alpha = ym / (1.f + x0 * x0);
  } else {
    beta = sxy / sxx;
    alpha = ym - beta * xm;
  }
  // unbiased residual variance (two-pass)
  float rm = 0.f;
  for (int i = 0; i < n; ++i) rm += ys[(size_t)i * C] - (alpha + beta * xs[(size_t)i * C]);
  rm /= (float)n;
  float rv = 0.f;
  for (int i = 0; i < n; ++i) {
    const float r = ys[(size_t)i * C] - (alpha + beta * xs[(size_t)i * C]) - rm;
    rv = fmaf(r, r, rv);
  }
  rv /= (float)(n - 1);
  alphas[id] = alpha;
  betas[id] = beta;
  inv_psi[id] = 1.f / rv;
  if (k == 0) {
    factor[2 * wdx] = xm;
    factor[2 * wdx + 1] = sxx / (float)(n - 1);
  }
}

}  // namespace

extern "C" int mta_dgp(uint64_t seed, int n_stocks, long n_samples, int mkt_df, float mkt_loc, float mkt_scale,
                       int idio_df, float idio_loc, float idio_scale, float a_loc, float a_scale, float b_loc,
                       float b_scale, float* r_market, float* r_stocks, float* alphas, float* betas, hipStream_t st) {
  const int maxdf = mkt_df > idio_df ? mkt_df : idio_df;
  // counter indices 2 * s * (df + 1) + 1 must fit 32 bits
  if (mkt_df < 1 || mkt_df > 64 || idio_df < 1 || idio_df > 64 ||
      n_samples >= (long)(4294967295UL / (2UL * (unsigned long)(maxdf + 1))))
    return 1;
  DgpArgs a{seed, n_stocks, n_samples, mkt_df, idio_df, mkt_loc, mkt_scale, idio_loc, idio_scale,
            a_loc, a_scale, b_loc, b_scale, r_market, r_stocks, alphas, betas};
  long blocks = (n_samples + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  dgp_market_kernel<<<(int)blocks, 256, 0, st>>>(a);
  long bx = (n_samples + 255) / 256;
  if (bx > 256) bx = 256;
  dgp_stocks_kernel<<<dim3((unsigned)bx, n_stocks), 256, 0, st>>>(a);
  return 0;
}

extern "C" void mta_ols_features(const float* target, int W, int K, int n, int C, float* alphas, float* betas,
                                 float* factor, float* inv_psi, hipStream_t st) {
  const long total = (long)W * K;
  ols_features_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>(target, W, K, n, C, alphas, betas, factor,
                                                                  inv_psi);
}
