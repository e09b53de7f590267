// fp32 RoPE self-attention for the transformer-encoder extra under trainer precision 32-true (ops/extras.py
// _TransformerEncoderF32Fn; the bf16 form is attention.hip).  Reference math: ops/extras.py attention_reference
// (RoPE on q and k, interleaved pairs (2i, 2i+1) at angle t * base^(-2i/HD); bidirectional softmax(q k^T / sqrt(HD)) v).
//
// One 256-thread workgroup per (sequence, head): the whole T <= 64 token problem lives in LDS as fp32 rows (stride
// HD + 1 / T + 1: conflict-free column walks; 35 / 51 / 83 KB of dynamic LDS for HD = 16 / 32 / 64), every product is an fp32 FMA loop on the VALU -- 2 x 64 x 64 x HD
// FLOP per (sequence, head), small next to the encoder's GEMMs -- so the scores, the softmax and both products are
// exact fp32, as the reference's fp32 graph.
//   forward : q, k rotated while staged; S = scale q k^T; P = softmax(S); O = P v; LSE saved per query row
//   backward: P recomputed from LSE; dV = P^T dO; dP = dO v^T; dS = P (dP - rowsum(dO o O)); dQ = scale dS k,
//             dK = scale dS^T q; the inverse rotation on dQ, dK; dqkv written [q | k | v] like qkv
// Layout: qkv [M][3D] fp32 with token row = seq * T + t, head h at columns h * HD of each third; out / dout [M][D];
// lse [nseq * heads][64].  RoPE (cos, sin) pairs come from the host-built table [T][HD/2] (bindings.cpp rope_table).
#include "common.h"

namespace {

constexpr int TMAX = 64;
constexpr int TPB = 256;

template <int HD>
struct AttnF32Smem {
  float q[TMAX][HD + 1], k[TMAX][HD + 1], v[TMAX][HD + 1], g[TMAX][HD + 1];  // g: dO (backward)
  float p[TMAX][TMAX + 1];
  float rowv[TMAX];  // backward: D_i = rowsum(dO o O)
};

struct AttnF32Args {
  const float* qkv;
  const float* out;   // backward: the forward output O
  const float* dout;  // backward: dO
  float* o;           // forward output
  float* lse;
  float* dqkv;
  const float2* rope;  // [T][HD/2] (cos, sin)
  int T, D, heads;
  float scale;
};

// q, k (rotated) and v rows of (sequence s, head h) into LDS
template <int HD>
__device__ __forceinline__ void stage_qkv(const AttnF32Args& a, int s, int h, AttnF32Smem<HD>& sm) {
  const int T = a.T, D = a.D;
  for (int e = threadIdx.x; e < T * (HD / 2); e += TPB) {
    const int t = e / (HD / 2), i = e % (HD / 2);
    const float* row = a.qkv + (size_t)(s * T + t) * 3 * D + h * HD + 2 * i;
    const float2 cs = a.rope[t * (HD / 2) + i];
    const float q0 = row[0], q1 = row[1], k0 = row[D], k1 = row[D + 1];
    sm.q[t][2 * i] = q0 * cs.x - q1 * cs.y;
    sm.q[t][2 * i + 1] = q0 * cs.y + q1 * cs.x;
    sm.k[t][2 * i] = k0 * cs.x - k1 * cs.y;
    sm.k[t][2 * i + 1] = k0 * cs.y + k1 * cs.x;
    sm.v[t][2 * i] = row[2 * D];
    sm.v[t][2 * i + 1] = row[2 * D + 1];
  }
}

template <int HD>
__global__ __launch_bounds__(TPB) void attention_f32_fwd_kernel(AttnF32Args a) {
  extern __shared__ __align__(16) char lds_raw[];
  AttnF32Smem<HD>& sm = *reinterpret_cast<AttnF32Smem<HD>*>(lds_raw);
  const int s = blockIdx.x / a.heads, h = blockIdx.x % a.heads;
  const int T = a.T, D = a.D;
  stage_qkv<HD>(a, s, h, sm);
  __syncthreads();
  for (int e = threadIdx.x; e < T * T; e += TPB) {
    const int i = e / T, j = e % T;
    float acc = 0.f;
#pragma unroll 8
    for (int c = 0; c < HD; ++c) acc = fmaf(sm.q[i][c], sm.k[j][c], acc);
    sm.p[i][j] = acc * a.scale;
  }
  __syncthreads();
  // softmax: four lanes per query row (T <= 64 rows x 4 = 256 threads)
  {
    const int i = threadIdx.x >> 2, part = threadIdx.x & 3;
    float m = -3.0e38f;
    if (i < T)
      for (int j = part; j < T; j += 4) m = fmaxf(m, sm.p[i][j]);
    m = fmaxf(m, __shfl_xor(m, 1));
    m = fmaxf(m, __shfl_xor(m, 2));
    float sum = 0.f;
    if (i < T)
      for (int j = part; j < T; j += 4) {
        const float ev = expf(sm.p[i][j] - m);
        sm.p[i][j] = ev;
        sum += ev;
      }
    sum += __shfl_xor(sum, 1);
    sum += __shfl_xor(sum, 2);
    if (i < T) {
      const float inv = 1.f / sum;
      for (int j = part; j < T; j += 4) sm.p[i][j] *= inv;
      if (part == 0) a.lse[(size_t)blockIdx.x * TMAX + i] = m + logf(sum);
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * HD; e += TPB) {
    const int i = e / HD, c = e % HD;
    float acc = 0.f;
    for (int j = 0; j < T; ++j) acc = fmaf(sm.p[i][j], sm.v[j][c], acc);
    a.o[(size_t)(s * T + i) * D + h * HD + c] = acc;
  }
}

template <int HD>
__global__ __launch_bounds__(TPB) void attention_f32_bwd_kernel(AttnF32Args a) {
  extern __shared__ __align__(16) char lds_raw[];
  AttnF32Smem<HD>& sm = *reinterpret_cast<AttnF32Smem<HD>*>(lds_raw);
  const int s = blockIdx.x / a.heads, h = blockIdx.x % a.heads;
  const int T = a.T, D = a.D;
  stage_qkv<HD>(a, s, h, sm);
  for (int e = threadIdx.x; e < T * HD; e += TPB) {
    const int t = e / HD, c = e % HD;
    sm.g[t][c] = a.dout[(size_t)(s * T + t) * D + h * HD + c];
  }
  // D_i = rowsum(dO o O): four lanes per row
  {
    const int i = threadIdx.x >> 2, part = threadIdx.x & 3;
    float acc = 0.f;
    if (i < T)
      for (int c = part; c < HD; c += 4) {
        const size_t o = (size_t)(s * T + i) * D + h * HD + c;
        acc = fmaf(a.dout[o], a.out[o], acc);
      }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (i < T && part == 0) sm.rowv[i] = acc;
  }
  __syncthreads();
  // P from the saved LSE
  for (int e = threadIdx.x; e < T * T; e += TPB) {
    const int i = e / T, j = e % T;
    float acc = 0.f;
#pragma unroll 8
    for (int c = 0; c < HD; ++c) acc = fmaf(sm.q[i][c], sm.k[j][c], acc);
    sm.p[i][j] = expf(acc * a.scale - a.lse[(size_t)blockIdx.x * TMAX + i]);
  }
  __syncthreads();
  float* dq = a.dqkv + (size_t)(s * T) * 3 * D + h * HD;
  // dV[j][c] = sum_i P[i][j] dO[i][c]
  for (int e = threadIdx.x; e < T * HD; e += TPB) {
    const int j = e / HD, c = e % HD;
    float acc = 0.f;
    for (int i = 0; i < T; ++i) acc = fmaf(sm.p[i][j], sm.g[i][c], acc);
    dq[(size_t)j * 3 * D + 2 * D + c] = acc;
  }
  // dS = P (dO v^T - D) in place of P (each entry read and written by its own thread, after dV read it)
  __syncthreads();
  for (int e = threadIdx.x; e < T * T; e += TPB) {
    const int i = e / T, j = e % T;
    float dp = 0.f;
#pragma unroll 8
    for (int c = 0; c < HD; ++c) dp = fmaf(sm.g[i][c], sm.v[j][c], dp);
    sm.p[i][j] = sm.p[i][j] * (dp - sm.rowv[i]);
  }
  __syncthreads();
  // dQ (rows of q) and dK (rows of k) by pairs, each rotated back: grad_in = R^T grad_out
  for (int e = threadIdx.x; e < 2 * T * (HD / 2); e += TPB) {
    const bool isk = e >= T * (HD / 2);
    const int r = isk ? e - T * (HD / 2) : e;
    const int t = r / (HD / 2), i = r % (HD / 2);
    float g0 = 0.f, g1 = 0.f;
    if (!isk) {
      for (int j = 0; j < T; ++j) {
        const float d = sm.p[t][j];
        g0 = fmaf(d, sm.k[j][2 * i], g0);
        g1 = fmaf(d, sm.k[j][2 * i + 1], g1);
      }
    } else {
      for (int j = 0; j < T; ++j) {
        const float d = sm.p[j][t];
        g0 = fmaf(d, sm.q[j][2 * i], g0);
        g1 = fmaf(d, sm.q[j][2 * i + 1], g1);
      }
    }
    g0 *= a.scale;
    g1 *= a.scale;
    const float2 cs = a.rope[t * (HD / 2) + i];
    float* dst = dq + (size_t)t * 3 * D + (isk ? D : 0) + 2 * i;
    dst[0] = g0 * cs.x + g1 * cs.y;
    dst[1] = g1 * cs.x - g0 * cs.y;
  }
}

}  // namespace

// bwd = 0: o, lse <- attention(qkv); bwd = 1: dqkv <- its backward (out = the forward's o, dout = dO).  Returns non-zero
// on an unsupported configuration (T > 64, head dim not 16 / 32 / 64).
extern "C" int mta_attention_f32(int bwd, const float* qkv, const float* out, const float* dout, float* o, float* lse,
                                 float* dqkv, int nseq, int T, int D, int heads, const float* rope, hipStream_t st) {
  if (T < 1 || T > TMAX || heads < 1 || D % heads || !rope || nseq < 1) return 1;
  const int HD = D / heads;
  AttnF32Args a{qkv, out, dout, o, lse, dqkv, reinterpret_cast<const float2*>(rope), T, D, heads,
                1.0f / sqrtf((float)HD)};
  const dim3 grid(nseq * heads), block(TPB);
#define ATTN_F32_CASE(HDV)                                                                                           \
  if (HD == HDV) {                                                                                                  \
    constexpr int bytes = (int)sizeof(AttnF32Smem<HDV>);                                                            \
    if (bytes > 65536) { /* gfx950: 160 KB of LDS per CU, opted into once per kernel */                            \
      static const bool attr =                                                                                      \
          hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_f32_fwd_kernel<HDV>),                        \
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess &&                   \
          hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_f32_bwd_kernel<HDV>),                        \
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess;                     \
      if (!attr) return 3;                                                                                          \
    }                                                                                                               \
    if (bwd) attention_f32_bwd_kernel<HDV><<<grid, block, bytes, st>>>(a);                                          \
    else attention_f32_fwd_kernel<HDV><<<grid, block, bytes, st>>>(a);                                              \
    return 0;                                                                                                       \
  }
  ATTN_F32_CASE(16)
  ATTN_F32_CASE(32)
  ATTN_F32_CASE(64)
#undef ATTN_F32_CASE
  return 2;
}
