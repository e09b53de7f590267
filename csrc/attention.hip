// Fused RoPE self-attention for the transformer-encoder extra (BASELINE.json north-star config 4).
//
// The encoder attends over one stock's lookback window: T <= 64 tokens, head dim HD in {32, 64}.  The
// whole (sequence, head) problem fits one wave: Q, K, V (64 x HD) and the 64 x 64 score tile live in LDS /
// VGPRs, so one 64-thread workgroup per (sequence, head) computes
//   forward : RoPE(q), RoPE(k) -> S = scale q k^T -> softmax (keys >= T masked) -> O = P V, LSE saved
//   backward: recompute P from LSE -> dV = P^T dO, dP = dO V^T, dS = P (dP - rowsum(dO o O)),
//             dQ = scale dS K, dK = dS^T (scale q) -> inverse RoPE on dQ, dK -> dqkv
// Every product is C = A B^T over k-contiguous LDS images (`mm`), so each v_mfma_f32_16x16x32_bf16
// operand is one ds_read_b128; transposed images are written once at load time (V^T, K^T, Q^T, dO^T) or
// straight from the accumulator layout (P^T, dS^T: four consecutive rows per lane = one 8-byte write).
// Layout: qkv [M][3*D] bf16 with token row = seq*T + t, columns [q | k | v], head h at h*HD.
// RoPE: interleaved pairs (2i, 2i+1), angle t * base^(-2i/HD), from a host-built (cos, sin) table [T][HD/2]
// (fp64-accurate; per-element sincosf/powf were ~1/4 of a launch).
// Four waves per (sequence, head): the q / k / v (/ dO) rows are loaded and rotated by one wave each, then wave w
// owns query tile w (scores, softmax, O; backward: P, dS) and token tile w (dV, dK, dQ): 4x the waves in flight
// of the one-wave form, which left the launch latency-bound (28 us per call at 416 workgroups, r2 trace).
#include "common.h"

namespace {

constexpr int TP = 64;        // padded tokens
constexpr int PLD = TP + 8;   // row stride of [.][64] images (bf16)

template <int HD>
struct AttnDims {
  static constexpr int RLD = HD + 8;  // row stride of [64][HD] images
};
// forward: q, k row-major (scores), V^T (B operand of O = P V), P
template <int HD>
struct FwdSmem : AttnDims<HD> {
  __bf16 q[TP * (HD + 8)], k[TP * (HD + 8)], vt[HD * PLD], p[TP * PLD];
  float rowv[TP];  // LSE
};
// backward: q, k (scores), v (dP), q^T (dK), k^T (dQ), dS / P^T / dS^T, dO and dO^T
template <int HD>
struct BwdSmem : AttnDims<HD> {
  __bf16 q[TP * (HD + 8)], k[TP * (HD + 8)], v[TP * (HD + 8)], qt[HD * PLD], kt[HD * PLD];
  __bf16 p[TP * PLD], pt[TP * PLD], dst[TP * PLD];
  __bf16 dO[TP * (HD + 8)], dOt[HD * PLD];
  float rowv[TP];  // D = rowsum(dO o O)
};

// C[16 x 16] += A[arow0 .. +16][0..K) * B[brow0 .. +16][0..K)^T, both k-contiguous LDS images
__device__ __forceinline__ f32x4 mm(const __bf16* A, int lda, int arow0, const __bf16* B, int ldb, int brow0,
                                   int K, f32x4 acc) {
  const int l = threadIdx.x & 63;
  for (int k0 = 0; k0 < K; k0 += 32) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + (arow0 + (l & 15)) * lda + k0 + 8 * (l >> 4));
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(B + (brow0 + (l & 15)) * ldb + k0 + 8 * (l >> 4));
    acc = mfma16x16x32(a, b, acc);
  }
  return acc;
}

// accumulator tile -> LDS: row-major (2-byte writes) or transposed (one 8-byte write per lane)
__device__ __forceinline__ void put_rows(__bf16* img, int ld, int row0, int col0, const f32x4& c) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < 4; ++r) img[(row0 + 4 * (l >> 4) + r) * ld + col0 + (l & 15)] = (__bf16)c[r];
}
__device__ __forceinline__ void put_cols(__bf16* img, int ld, int row0, int col0, const f32x4& c) {
  const int l = threadIdx.x & 63;
  bf16x4 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = (__bf16)c[r];
  *reinterpret_cast<bf16x4*>(img + (col0 + (l & 15)) * ld + row0 + 4 * (l >> 4)) = v;
}

struct AttnArgs {
  const __bf16* qkv;
  __bf16* out;       // [M][D]
  float* lse;        // [nseq * heads][TP]
  const __bf16* dout;
  // backward with the output projection's input gradient fused in (dout null): dO = dX1 Wo, dX1 [M][D] bf16 rows,
  // Wo^T as a fragment-major image (csrc/tr_ffn.hip frag_pack, transposed)
  const __bf16* dx1;
  const __bf16* wot;
  __bf16* dqkv;      // [M][3D]
  int T, D, heads;
  float scale, rope_base;
  const float* rope;  // [T][HD/2] (cos, sin) pairs
};

// load this (seq, head)'s q, k, v rows (lane = token), apply RoPE (and the softmax scale to q), and write
// the requested row-major (rm[i]) and transposed (tr[i]) images (nullptr = not needed)
template <int HD>
__device__ __forceinline__ void load_qkv(const AttnArgs& a, int seq, int h, __bf16* const rm[3], __bf16* const tr[3],
                                         int only) {
  constexpr int RLD = HD + 8;
  const int t = threadIdx.x & 63;
  const bool ok = t < a.T;
  const size_t row = (size_t)seq * a.T + (ok ? t : 0);
  const __bf16* base = a.qkv + row * 3 * a.D + h * HD;
  const float2* rope = reinterpret_cast<const float2*>(a.rope) + (size_t)(ok ? t : 0) * (HD / 2);
#pragma unroll
  for (int which = 0; which < 3; ++which) {
    if (which != only || (!rm[which] && !tr[which])) continue;
    float x[HD];
#pragma unroll
    for (int c = 0; c < HD; c += 8) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(base + which * a.D + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[c + j] = ok ? (float)v[j] : 0.f;
    }
    if (which < 2) {
#pragma unroll
      for (int i = 0; i < HD / 2; ++i) {
        const float2 r = rope[i];
        const float cs = r.x, sn = r.y;
        const float x0 = x[2 * i], x1 = x[2 * i + 1];
        x[2 * i] = x0 * cs - x1 * sn;
        x[2 * i + 1] = x0 * sn + x1 * cs;
      }
      if (which == 0) {
#pragma unroll
        for (int c = 0; c < HD; ++c) x[c] *= a.scale;
      }
    }
    if (rm[which]) {
#pragma unroll
      for (int c = 0; c < HD; c += 8) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (__bf16)x[c + j];
        *reinterpret_cast<bf16x8*>(rm[which] + t * RLD + c) = v;
      }
    }
    if (tr[which]) {
#pragma unroll
      for (int c = 0; c < HD; ++c) tr[which][c * PLD + t] = (__bf16)x[c];
    }
  }
}

// S tile (qi, ki) with keys >= T masked
template <int HD, class S>
__device__ __forceinline__ f32x4 score_tile(const S& s, int qi, int ki, int T) {
  f32x4 acc = mm(s.q, HD + 8, 16 * qi, s.k, HD + 8, 16 * ki, HD, f32x4{0.f, 0.f, 0.f, 0.f});
  const int key = 16 * ki + ((threadIdx.x & 63) & 15);
  if (key >= T) acc = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  return acc;
}

template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  FwdSmem<HD>& s = *reinterpret_cast<FwdSmem<HD>*>(smem_raw);
  const int seq = blockIdx.x / a.heads, h = blockIdx.x % a.heads;
  const int l = threadIdx.x & 63, wave = threadIdx.x >> 6;
  {
    __bf16* const rm[3] = {s.q, s.k, nullptr};
    __bf16* const tr[3] = {nullptr, nullptr, s.vt};
    load_qkv<HD>(a, seq, h, rm, tr, wave);  // wave 0: q, 1: k, 2: v^T
  }
  __syncthreads();
  // scores + softmax of query tile qi = wave, P -> LDS (row-major, the A operand of O = P V)
  {
    const int qi = wave;
    f32x4 sc[4];
#pragma unroll
    for (int ki = 0; ki < 4; ++ki) sc[ki] = score_tile<HD>(s, qi, ki, a.T);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float m = fmaxf(fmaxf(sc[0][r], sc[1][r]), fmaxf(sc[2][r], sc[3][r]));
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
      float sum = 0.f;
#pragma unroll
      for (int ki = 0; ki < 4; ++ki) {
        sc[ki][r] = __expf(sc[ki][r] - m);
        sum += sc[ki][r];
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) sum += __shfl_xor(sum, off, 64);
      const float inv = 1.0f / sum;
#pragma unroll
      for (int ki = 0; ki < 4; ++ki) sc[ki][r] *= inv;
      if ((l & 15) == 0) s.rowv[16 * qi + 4 * (l >> 4) + r] = m + __logf(sum);
    }
#pragma unroll
    for (int ki = 0; ki < 4; ++ki) put_rows(s.p, PLD, 16 * qi, 16 * ki, sc[ki]);
  }
  __syncthreads();
  // O = P V  (B = V^T rows = features, k = tokens) for query tile qi = wave
  const size_t seqrow = (size_t)seq * a.T;
  {
    const int qi = wave;
#pragma unroll
    for (int dj = 0; dj < HD / 16; ++dj) {
      const f32x4 o = mm(s.p, PLD, 16 * qi, s.vt, PLD, 16 * dj, TP, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * qi + 4 * (l >> 4) + r;
        if (t < a.T) a.out[(seqrow + t) * a.D + h * HD + 16 * dj + (l & 15)] = (__bf16)o[r];
      }
    }
  }
  if (wave == 0) a.lse[(size_t)blockIdx.x * TP + l] = s.rowv[l];
}

// B fragment (16 output features n0.., 32 k from k0) of a fragment-major [N][K] image: 1 KB contiguous per wave
__device__ __forceinline__ bf16x8 fm_frag(const __bf16* w, int K, int n0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(w + ((size_t)((n0 >> 4) * (K >> 5) + (k0 >> 5)) << 9) + 8 * lane);
}

template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_kernel(AttnArgs a) {
  constexpr int RLD = HD + 8;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  BwdSmem<HD>& s = *reinterpret_cast<BwdSmem<HD>*>(smem_raw);
  const int seq = blockIdx.x / a.heads, h = blockIdx.x % a.heads;
  const int l = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t seqrow0 = (size_t)seq * a.T;
  auto put_dO = [&](int tt, const f32x4* acc) {
#pragma unroll
    for (int dj = 0; dj < HD / 16; ++dj) {
      f32x4 rb;  // rounded as the unfused chain's bf16 dO tensor
#pragma unroll
      for (int r = 0; r < 4; ++r) rb[r] = (float)(__bf16)acc[dj][r];
      put_rows(s.dO, RLD, 16 * tt, 16 * dj, rb);
      put_cols(s.dOt, PLD, 16 * tt, 16 * dj, rb);
    }
  };
  // wave 3 (after dO is in LDS): D = rowsum(dO o O), token t = lane
  auto dO_rowsum = [&]() {
    const int t = l;
    const bool ok = t < a.T;
    const __bf16* osrc = a.out + (seqrow0 + (ok ? t : 0)) * a.D + h * HD;
    float dsum = 0.f;
#pragma unroll
    for (int c = 0; c < HD; c += 8) {
      const bf16x8 dv = *reinterpret_cast<const bf16x8*>(s.dO + t * RLD + c);
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(osrc + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum += ok ? (float)dv[j] * (float)ov[j] : 0.f;
    }
    s.rowv[t] = dsum;
  };
  if (wave < 3) {
    __bf16* const rm[3] = {s.q, s.k, s.v};
    __bf16* const tr[3] = {s.qt, s.kt, nullptr};
    load_qkv<HD>(a, seq, h, rm, tr, wave);  // wave 0: q, q^T; 1: k, k^T; 2: v
  }
  if (a.dx1 && a.D <= 4 * 32) {
    // this head's dO = dX1 rows . Wo^T[head features] (64 x HD, K = D <= 128: the transformer's 4 heads of 32) on
    // the matrix cores -- the output projection's input-gradient GEMM, fused: every wave one 16-token tile, its W_o^T
    // fragments and dX1 row pieces issued together (one wave doing all four tiles, one load round trip per k-step, was
    // the kernel's critical path at B >= 8), then D = rowsum(dO o O) after a barrier
    {
      const int tt = wave;
      const int t = 16 * tt + (l & 15);
      const bool ok = t < a.T;
      const __bf16* arow = a.dx1 + (seqrow0 + (ok ? t : 0)) * a.D + 8 * (l >> 4);
      bf16x8 wf[4][HD / 16], af[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        af[kk] = ok && 32 * kk < a.D ? *reinterpret_cast<const bf16x8*>(arow + 32 * kk) : bf16x8{};
#pragma unroll
        for (int dj = 0; dj < HD / 16; ++dj)
          wf[kk][dj] = 32 * kk < a.D ? fm_frag(a.wot, a.D, h * HD + 16 * dj, 32 * kk, l) : bf16x8{};
      }
      f32x4 acc[HD / 16];
#pragma unroll
      for (int dj = 0; dj < HD / 16; ++dj) acc[dj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int dj = 0; dj < HD / 16; ++dj) acc[dj] = mfma16x16x32(af[kk], wf[kk][dj], acc[dj]);
      put_dO(tt, acc);
    }
    __syncthreads();  // dO complete
    if (wave == 3) dO_rowsum();
  } else if (wave == 3 && a.dx1) {
    // wider D: wave 3 alone, one k-step at a time
#pragma unroll 1
    for (int tt = 0; tt < TP / 16; ++tt) {
      f32x4 acc[HD / 16];
#pragma unroll
      for (int dj = 0; dj < HD / 16; ++dj) acc[dj] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int t = 16 * tt + (l & 15);
      const bool ok = t < a.T;
      const __bf16* arow = a.dx1 + (seqrow0 + (ok ? t : 0)) * a.D + 8 * (l >> 4);
#pragma unroll 1
      for (int k0 = 0; k0 < a.D; k0 += 32) {
        bf16x8 af = *reinterpret_cast<const bf16x8*>(arow + k0);
        if (!ok) af = bf16x8{};
#pragma unroll
        for (int dj = 0; dj < HD / 16; ++dj) acc[dj] = mfma16x16x32(af, fm_frag(a.wot, a.D, h * HD + 16 * dj, k0, l), acc[dj]);
      }
      put_dO(tt, acc);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's dO rows are in LDS for its own lanes
    dO_rowsum();
  } else if (wave == 3) {
    // wave 3: dO rows (row-major + transposed) and D = rowsum(dO o O)
    const int t = l;
    const bool ok = t < a.T;
    const size_t row = (size_t)seq * a.T + (ok ? t : 0);
    const __bf16* dsrc = a.dout + row * a.D + h * HD;
    const __bf16* osrc = a.out + row * a.D + h * HD;
    float dsum = 0.f;
#pragma unroll
    for (int c = 0; c < HD; c += 8) {
      const bf16x8 dv = *reinterpret_cast<const bf16x8*>(dsrc + c);
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(osrc + c);
      bf16x8 w;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = ok ? (float)dv[j] : 0.f;
        dsum += d * (ok ? (float)ov[j] : 0.f);
        w[j] = (__bf16)d;
        s.dOt[(c + j) * PLD + t] = (__bf16)d;
      }
      *reinterpret_cast<bf16x8*>(s.dO + t * RLD + c) = w;
    }
    s.rowv[t] = dsum;
  }
  const float* lse = a.lse + (size_t)blockIdx.x * TP;
  __syncthreads();
  // P (recomputed), dS = P (dP - D)  ->  P^T, dS, dS^T images, query tile qi = wave
  {
    const int qi = wave;
    float lrow[4], drow[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = 16 * qi + 4 * (l >> 4) + r;
      lrow[r] = lse[q];
      drow[r] = s.rowv[q];
    }
#pragma unroll
    for (int ki = 0; ki < 4; ++ki) {
      f32x4 p = score_tile<HD>(s, qi, ki, a.T);
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] = __expf(p[r] - lrow[r]);
      const f32x4 dp = mm(s.dO, RLD, 16 * qi, s.v, RLD, 16 * ki, HD, f32x4{0.f, 0.f, 0.f, 0.f});
      f32x4 ds;
#pragma unroll
      for (int r = 0; r < 4; ++r) ds[r] = p[r] * (dp[r] - drow[r]);
      put_cols(s.pt, PLD, 16 * qi, 16 * ki, p);    // P^T  [key][query]
      put_rows(s.p, PLD, 16 * qi, 16 * ki, ds);    // dS   [query][key]
      put_cols(s.dst, PLD, 16 * qi, 16 * ki, ds);  // dS^T [key][query]
    }
  }
  __syncthreads();
  // dV = P^T dO, dK = dS^T (scale q), dQ = scale dS K; inverse RoPE on dQ / dK; write dqkv
  const size_t seqrow = (size_t)seq * a.T;
  const int col = l & 15;
  {
    const int ti = wave;  // token tile
#pragma unroll
    for (int dj = 0; dj < HD / 16; ++dj) {
      const f32x4 dv = mm(s.pt, PLD, 16 * ti, s.dOt, PLD, 16 * dj, TP, f32x4{0.f, 0.f, 0.f, 0.f});
      f32x4 dk = mm(s.dst, PLD, 16 * ti, s.qt, PLD, 16 * dj, TP, f32x4{0.f, 0.f, 0.f, 0.f});
      f32x4 dq = mm(s.p, PLD, 16 * ti, s.kt, PLD, 16 * dj, TP, f32x4{0.f, 0.f, 0.f, 0.f});
      const int c = 16 * dj + col;       // feature index; RoPE pair (c & ~1, c | 1) sits in lanes l, l^1
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * ti + 4 * (l >> 4) + r;
        const float2 rr = reinterpret_cast<const float2*>(a.rope)[(size_t)(t < a.T ? t : 0) * (HD / 2) + (c >> 1)];
        const float cs = rr.x, sn = rr.y;
        const float pq = __shfl_xor(dq[r], 1, 64), pk = __shfl_xor(dk[r], 1, 64);
        // forward: y0 = x0 c - x1 s, y1 = x0 s + x1 c  =>  dx0 = dy0 c + dy1 s, dx1 = -dy0 s + dy1 c
        const float gq = (c & 1) ? (-pq * sn + dq[r] * cs) : (dq[r] * cs + pq * sn);
        const float gk = (c & 1) ? (-pk * sn + dk[r] * cs) : (dk[r] * cs + pk * sn);
        if (t < a.T) {
          __bf16* o = a.dqkv + (seqrow + t) * 3 * a.D + h * HD + c;
          o[0] = (__bf16)(gq * a.scale);
          o[a.D] = (__bf16)gk;
          o[2 * a.D] = (__bf16)dv[r];
        }
      }
    }
  }
}

}  // namespace

extern "C" int mta_attention(int bwd, const void* qkv, void* out, float* lse, const void* dout, void* dqkv, int nseq,
                             int T, int D, int heads, float rope_base, const float* rope, const void* dx1,
                             const void* wot, hipStream_t st) {
  if (T < 1 || T > TP || D % heads || !rope) return 1;
  if (bwd && !dout && !(dx1 && wot && D % 32 == 0)) return 4;
  const int HD = D / heads;
  AttnArgs a;
  a.qkv = static_cast<const __bf16*>(qkv);
  a.out = static_cast<__bf16*>(out);
  a.lse = lse;
  a.dout = static_cast<const __bf16*>(dout);
  a.dx1 = dout ? nullptr : static_cast<const __bf16*>(dx1);
  a.wot = static_cast<const __bf16*>(wot);
  a.dqkv = static_cast<__bf16*>(dqkv);
  a.T = T;
  a.D = D;
  a.heads = heads;
  a.scale = 1.0f / sqrtf((float)HD);
  a.rope_base = rope_base;
  a.rope = rope;
  const int blocks = nseq * heads;
  if (HD == 32) {
    if (bwd) attn_bwd_kernel<32><<<blocks, 256, sizeof(BwdSmem<32>), st>>>(a);
    else attn_fwd_kernel<32><<<blocks, 256, sizeof(FwdSmem<32>), st>>>(a);
  } else if (HD == 64) {
    // > 64 KB of dynamic LDS (gfx950 has 160 KB per CU): opt in once per kernel
    static bool attr = false;
    if (!attr) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_kernel<64>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(BwdSmem<64>)) != hipSuccess)
        return 3;
      attr = true;
    }
    if (bwd) attn_bwd_kernel<64><<<blocks, 256, sizeof(BwdSmem<64>), st>>>(a);
    else attn_fwd_kernel<64><<<blocks, 256, sizeof(FwdSmem<64>), st>>>(a);
  } else {
    return 2;
  }
  return 0;
}
