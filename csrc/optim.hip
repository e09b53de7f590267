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

extern "C" void mta_scale(float* x, long n, float s, hipStream_t st) {
  const long n4 = n / 4;
  scale_kernel<<<grid_for(n4), TPB, 0, st>>>(reinterpret_cast<float4*>(x), n4, s);
}
