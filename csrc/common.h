// Shared device helpers for the masters_thesis_amd CDNA4 (gfx950) kernels.
//
// Everything here is written for MI355X directly: wave64, MFMA fragments of
// v_mfma_f32_16x16x32_bf16 / v_mfma_f32_16x16x4_f32, bf16 round-to-nearest-even
// conversion via the __bf16 type (lowers to v_cvt_pk_bf16_f32 on gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "batch_gather.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
// LDS destination of global_load_lds (LDS-DMA: 16 B per lane at the wave-uniform base + 16 lane, no VGPR round trip)
typedef __attribute__((address_space(3))) void lds_void;
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Matmul precision for fp32 recurrences, mirroring torch.set_float32_matmul_precision:
//   PREC_F32    'highest' : exact f32-input MFMA (v_mfma_f32_16x16x4_f32, fmaf-chain numerics)
//   PREC_BF16X3 'bf16x3'  : x = hi + lo split into two bf16, a*b ~= hi*hi + hi*lo + lo*hi (3 bf16 MFMAs,
//                           ~16 mantissa bits per product, fp32 accumulate; > TF32, which cuDNN uses)
//   PREC_BF16   'medium'  : single bf16 MFMA pass, fp32 accumulate (the reference's own setting,
//                           train.py:13 set_float32_matmul_precision('medium'))
//   PREC_F16X2  'high'    : LSTM forward only -- the activation operand (|h| < 1, |dropout(h)| < 1.5) as ONE fp16
//                           (11-bit significand = TF32's), the weight as fp16 hi + lo (~22 bits): a*w ~= a*hi + a*lo,
//                           2 f16 MFMAs instead of 3 bf16 ones.  TF32-class, i.e. what cuDNN's LSTM runs for the
//                           reference by default (cudnn.allow_tf32), with the weights more exact than TF32's
enum { PREC_F32 = 0, PREC_BF16X3 = 1, PREC_BF16 = 2, PREC_F16X2 = 3 };

// Activations on the transcendental unit: v_exp_f32 + v_rcp_f32 (1 ulp) instead of the ~10-instruction
// IEEE division sequence a plain '1.0f / x' compiles to.
__device__ __forceinline__ float mta_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
// exp(-x) as v_exp_f32 (2^y) of one product: -log2(e) and -2 log2(e) folded into one constant each (hipcc keeps
// `-2 * x` and the log2(e) scale of __expf as two multiplies: 8 extra VALU per LSTM step and lane)
__device__ __forceinline__ float mta_sigmoid(float x) {
  return mta_rcp(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
__device__ __forceinline__ float mta_tanh(float x) {
  // 2*sigmoid(2x) - 1: saturates cleanly at +-1
  return fmaf(2.0f, mta_rcp(1.0f + __builtin_amdgcn_exp2f(x * -2.8853900817779268f)), -1.0f);
}

__device__ __forceinline__ void split_bf16(float x, __bf16& hi, __bf16& lo) {
  hi = (__bf16)x;
  lo = (__bf16)(x - (float)hi);
}

__device__ __forceinline__ void split_bf16(float x, _Float16& hi, _Float16& lo) {  // fp16 hi + lo (PREC_F16X2)
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16x16x32(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16x16x4f32(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Wave-level sum (64 lanes) via DPP-friendly shuffles.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Wave sums on the DPP path (no LDS round trip per step, unlike __shfl_xor -> ds_bpermute): two quad_perm
// and two row_shr steps reduce each 16-lane row (the row total lands in its lane 15), the four row totals
// are read as scalars.  Every lane of the wave must be active (all call sites run whole waves).
template <int CTRL>
__device__ __forceinline__ int mta_dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);  // invalid source lane -> 0
}
template <int CTRL>
__device__ __forceinline__ float mta_dpp(float v) {
  return __builtin_bit_cast(float, mta_dpp_i<CTRL>(__builtin_bit_cast(int, v)));
}
template <int CTRL>
__device__ __forceinline__ double mta_dpp(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const unsigned lo = (unsigned)mta_dpp_i<CTRL>((int)(b & 0xffffffffll));
  const unsigned hi = (unsigned)mta_dpp_i<CTRL>((int)(b >> 32));
  return __builtin_bit_cast(double, (long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ float mta_readlane(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}
__device__ __forceinline__ double mta_readlane(double v, int lane) {
  const long long b = __builtin_bit_cast(long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)hi << 32) | lo));
}
template <typename T>
__device__ __forceinline__ T wave_sum_dpp(T v) {
  v += mta_dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += mta_dpp<0x4E>(v);   // quad_perm [2,3,0,1]: every lane holds its quad's sum
  v += mta_dpp<0x114>(v);  // row_shr:4
  v += mta_dpp<0x118>(v);  // row_shr:8: lane 15 of each row holds the row's sum
  return (mta_readlane(v, 15) + mta_readlane(v, 31)) + (mta_readlane(v, 47) + mta_readlane(v, 63));
}

// Block-level sum for blockDim.x <= 1024; `scratch` needs blockDim.x/64 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

// s_waitcnt vmcnt(0) as a builtin (the compiler's waitcnt pass sees it, unlike inline asm).
// gfx9 encoding: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt[5:4]=0  ->  0x0F70
__device__ __forceinline__ void mta_wait_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// s_waitcnt vmcnt(N): all but the N most recently issued vector-memory ops have completed (gfx9 returns
// them in issue order); expcnt / lgkmcnt not waited on
template <int N>
__device__ __forceinline__ void mta_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}

// GELU (erf form, torch.nn.GELU() default) and its derivative.
// erf(x / sqrt 2) for the exact (erf) GELU: Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7) on |z|, one exp (shared
// with the GELU derivative's density) and one rcp instead of the library erff's branchy ~40-instruction sequence --
// the GELU epilogue of the mlp_large forward GEMM was ~15 % of that kernel (r3 GEMM probe, epi=1 vs plain)
__device__ __forceinline__ float mta_erf_sqrt1_2(float x, float e /* = exp(-x*x/2) */) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float p = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                           0.254829592f);
  return copysignf(1.0f - p * e, x);
}
__device__ __forceinline__ float mta_gelu(float x) {
  return 0.5f * x * (1.0f + mta_erf_sqrt1_2(x, __expf(-0.5f * x * x)));
}
__device__ __forceinline__ float mta_gelu_grad(float x) {
  const float e = __expf(-0.5f * x * x);
  return 0.5f * (1.0f + mta_erf_sqrt1_2(x, e)) + x * 0.3989422804014327f * e;
}
// both, sharing the exp and the erf (the norm backward that recomputes the GELU output from its input)
__device__ __forceinline__ void mta_gelu_and_grad(float x, float& g, float& gp) {
  const float e = __expf(-0.5f * x * x);
  const float phi = 0.5f * (1.0f + mta_erf_sqrt1_2(x, e));
  g = x * phi;
  gp = phi + x * 0.3989422804014327f * e;
}

// Counter-based dropout: keep(seed, row, col) from a stateless 32-bit hash (murmur3-style finaliser of
// two rounds), so forward and backward regenerate the same mask without storing it and a captured
// graph only needs the device-resident seed advanced once per step.
__device__ __forceinline__ uint32_t mta_hash3(uint64_t seed, uint32_t a, uint32_t b) {
  uint32_t h = (uint32_t)seed ^ 0x9E3779B9u;
  uint32_t k[3] = {(uint32_t)(seed >> 32), a, b};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    uint32_t x = k[i] * 0xCC9E2D51u;
    x = (x << 15) | (x >> 17);
    x *= 0x1B873593u;
    h ^= x;
    h = (h << 13) | (h >> 19);
    h = h * 5u + 0xE6546B64u;
  }
  h ^= 12u;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
// Cheaper dropout for hot recurrences: ONE lowbias32-style hash per (row pair, column) gives two 16-bit uniforms
// (p resolved to 1/65536): 3 multiplies per two elements instead of mta_hash3's ~8 per element.  Row pair = row >> 1,
// element e = row & 1 takes bits [16 e, 16 e + 16).  seed / column parts are loop-invariant (hoisted by callers).
__device__ __forceinline__ uint32_t mta_pair_seed(uint64_t seed) {
  return (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x27D4EB2Fu);
}
__device__ __forceinline__ uint32_t mta_pair_col(uint32_t col) {
  const uint32_t b = col * 0x85EBCA77u;
  return (b << 13) | (b >> 19);
}
__device__ __forceinline__ uint32_t mta_pair_hash(uint32_t pseed, uint32_t pair, uint32_t pcol) {
  uint32_t x = pseed ^ (pair * 0x9E3779B1u) ^ pcol;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool mta_pair_keep(uint32_t hash, int e, float p) {
  return (float)((hash >> (16 * e)) & 0xFFFFu) * (1.0f / 65536.0f) >= p;
}
// Dropout scales (0 or 1/(1-p)) of the 4 consecutive columns c .. c+3 (c % 4 == 0) of one row: two lowbias32-style
// hashes of (row, column pair) give the four 16-bit uniforms (p resolved to 1/65536) -- 2 quarter-rate integer
// multiplies per element instead of mta_hash3's ~8, which made the wide LayerNorm forward VALU-bound.  The norm
// kernels' dropout, forward and backward alike.
__device__ __forceinline__ void mta_dropout_scale4(uint64_t seed, uint32_t row, uint32_t c, float p, float (&s)[4]) {
  const uint32_t ps = mta_pair_seed(seed);
  const uint32_t thr = (uint32_t)(p * 65536.f + 0.5f);
  const float sc = 1.0f / (1.0f - p);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t x = mta_pair_hash(ps, row, mta_pair_col((c >> 1) + h));
    s[2 * h] = (x & 0xFFFFu) >= thr ? sc : 0.f;
    s[2 * h + 1] = (x >> 16) >= thr ? sc : 0.f;
  }
}
// 0 or 1/(1-p)
__device__ __forceinline__ float mta_dropout_scale(uint64_t seed, uint32_t row, uint32_t col, float p) {
  const float u = (float)(mta_hash3(seed, row, col) >> 8) * (1.0f / 16777216.0f);
  return u >= p ? 1.0f / (1.0f - p) : 0.0f;
}
