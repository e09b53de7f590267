// One launch per transformer-encoder block forward (BASELINE.json north-star config 4: d = 128, 4 heads of 32,
// FFN 512, RMSNorm, RoPE self-attention over a T <= 64 token window).
//
// The unfused forward is 7 launches per block (norm, QKV GEMM, attention, proj GEMM, norm, FFN-up GEMM, FFN-down
// GEMM), each a 6,000 x 128-ish problem that is launch/latency bound (8-11 us per GEMM at 25-75 TFLOP/s, r3
// transformer trace).  Here one 256-thread workgroup owns one sequence (T tokens padded to 64 rows; wave w owns
// token rows 16w .. 16w+15) and runs the whole block with every activation in LDS / registers:
//   xn  = RMSNorm1(x)                       (x rows from global, rstd r1 saved)
//   qkv = xn Wqkv^T + bqkv                  (bf16, saved UNROTATED for the attention backward)
//   o   = softmax(RoPE(q) RoPE(k)^T / sqrt(32), keys >= T masked) v      per head (LSE saved)
//   x1  = x + o Wo^T + bo                   (fp32, saved)
//   xn2 = RMSNorm2(x1)                      (bf16 + r2 saved)
//   u   = dropout(GELU(xn2 W1^T + b1))      (pre-activation and u saved, bf16; the GEMM epilogue's pair hash)
//   x2  = x1 + u W2^T + b2                  (fp32: the next block's input)
// writing exactly the tensors the unfused forward saves, so the (unchanged) backward consumes them as before.
// Weights (384 KB per block, L2-resident across the 100+ workgroups) stream through two 34-KB LDS buffers in
// [128 rows][128 k] chunks: Wq, Wk, Wv, Wo, (W1_c, W2_c) x 4, the next chunk's global loads issued into registers
// before the current chunk's MFMAs.  Every product is C = A B^T over k-contiguous LDS images with 272-byte rows
// (conflict-free ds_read_b128 fragments), v_mfma_f32_16x16x32_bf16.
// Reference semantics: the PyTorch encoder block of models/extras.py (transformer_reference), the unfused kernel
// chain of ops/extras.py._TransformerEncoderFn.forward.
#include "common.h"

namespace {

constexpr int TD = 128, TFF = 512, THD = 32, TROWS = 64, TLD = TD + 8;  // image row stride (bf16): 272 B
constexpr int PLD2 = TROWS + 8;                                         // [.][64] images (V^T, P)
constexpr int WCHUNK = 128 * TLD;                                       // one weight chunk image (bf16 elements)

struct TrLayerArgs {
  const float* xs;                        // [M][128] block input
  const __bf16 *wqkv, *wo, *w1, *w2;      // [384][128], [128][128], [512][128], [128][512]
  const float *g1, *bqkv, *bo, *g2, *b1, *b2;
  float eps;
  __bf16 *xn, *qkv, *o, *xn2, *pre1, *u;  // saved activations
  float *x1, *x2, *r1, *r2, *lse;         // lse: [nseq * heads][64]
  const float* rope;                      // [T][16] (cos, sin)
  const uint64_t* seed;                   // FFN dropout seed (device scalar) or null
  float drop_p;
  int T;
};

struct TrSmem {
  __bf16 w[2][WCHUNK];      // weight chunk ping-pong
  __bf16 a[TROWS * TLD];    // xn -> o -> xn2 (A operands)
  __bf16 q[TROWS * TLD];    // RoPE'd, scaled q (all heads) -> u chunk during the FFN
  __bf16 k[TROWS * TLD];    // RoPE'd k
  __bf16 vt[TD * PLD2];     // V^T [feature][token]
  __bf16 p[TROWS * PLD2];   // softmax probabilities of the current head (wave w: rows 16w..)
  float prm[1408];          // g1 | bqkv | bo | g2 | b1 | b2: read from LDS, never from global after a store
};
// offsets into TrSmem::prm
constexpr int P_G1 = 0, P_BQKV = 128, P_BO = 512, P_G2 = 640, P_B1 = 768, P_B2 = 1280;

// C[16 x 16] += A[arow0 .. +16][k0 .. k0+K) * B[brow0 .. +16][k0 .. k0+K)^T over k-contiguous LDS images
__device__ __forceinline__ f32x4 mm16(const __bf16* A, int lda, int arow0, const __bf16* B, int ldb, int brow0,
                                      int k0, int K, f32x4 acc) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int kk = 0; kk < K; kk += 32) {
    const bf16x8 av = *reinterpret_cast<const bf16x8*>(A + (arow0 + (l & 15)) * lda + k0 + kk + 8 * (l >> 4));
    const bf16x8 bv = *reinterpret_cast<const bf16x8*>(B + (brow0 + (l & 15)) * ldb + k0 + kk + 8 * (l >> 4));
    acc = mfma16x16x32(av, bv, acc);
  }
  return acc;
}

// A fragments of this wave's 16 rows over k = 0..127 of an image (4 x ds_read_b128, loaded once per phase)
__device__ __forceinline__ void afrags(const __bf16* A, int lda, int arow0, bf16x8 (&af)[4]) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 4; ++k) af[k] = *reinterpret_cast<const bf16x8*>(A + (arow0 + (l & 15)) * lda + 32 * k + 8 * (l >> 4));
}
// acc[nt] (+)= A(16 rows x 128) B[16 nt .. 16 nt + 15][0..127]^T for nt = 0..7, every B read issued ahead of the
// MFMAs that use it (one wave per SIMD here: a read -> MFMA chain per tile exposed the LDS latency on every MFMA)
__device__ __forceinline__ void rowblock(const bf16x8 (&af)[4], const __bf16* B, f32x4 (&acc)[8]) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int nt = 0; nt < 8; nt += 2) {
    bf16x8 b0[4], b1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      b0[k] = *reinterpret_cast<const bf16x8*>(B + (16 * nt + (l & 15)) * TLD + 32 * k + 8 * (l >> 4));
      b1[k] = *reinterpret_cast<const bf16x8*>(B + (16 * nt + 16 + (l & 15)) * TLD + 32 * k + 8 * (l >> 4));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[nt] = mfma16x16x32(af[k], b0[k], acc[nt]);
      acc[nt + 1] = mfma16x16x32(af[k], b1[k], acc[nt + 1]);
    }
  }
}

// weight chunk c of the block's sequence: rows/cols of a [128 x 128] slice of one matrix
struct Chunk {
  const __bf16* base;
  int ld;
};
__device__ __forceinline__ Chunk chunk_of(const TrLayerArgs& a, int c) {
  if (c < 3) return Chunk{a.wqkv + (size_t)c * 128 * TD, TD};  // Wq, Wk, Wv
  if (c == 3) return Chunk{a.wo, TD};
  const int f = (c - 4) >> 1;
  if (((c - 4) & 1) == 0) return Chunk{a.w1 + (size_t)f * 128 * TD, TD};  // W1 rows f*128 ..
  return Chunk{a.w2 + f * 128, TFF};                                     // W2 columns f*128 ..
}
constexpr int NCHUNKS = 12;

__device__ __forceinline__ void chunk_load(const TrLayerArgs& a, int c, uint4 (&r)[8]) {
  const Chunk ch = chunk_of(a, c);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int idx = threadIdx.x + 256 * i, row = idx >> 4, kc = idx & 15;
    r[i] = *reinterpret_cast<const uint4*>(ch.base + (size_t)row * ch.ld + 8 * kc);
  }
}
__device__ __forceinline__ void chunk_store(__bf16* w, const uint4 (&r)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int idx = threadIdx.x + 256 * i, row = idx >> 4, kc = idx & 15;
    *reinterpret_cast<uint4*>(w + row * TLD + 8 * kc) = r[i];
  }
}

__device__ __forceinline__ uint32_t tr_pair_hash(uint32_t s, uint32_t mpair, uint32_t n) {
  const uint32_t b = n * 0x85EBCA77u;  // == gemm.hip gemm_pair_hash: the backward GEMM regenerates this mask
  uint32_t x = s ^ (mpair * 0x9E3779B1u) ^ ((b << 13) | (b >> 19));
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

#ifdef MTA_TR_STAMPS
__device__ unsigned long long tr_stamp[16];  // phase durations summed over workgroups (wave 0, lane 0)
#define TSTAMP(i)                                                                       \
  do {                                                                                  \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                       \
    if (tid == 0) atomicAdd(&tr_stamp[i], now_ - t_prev_);                              \
    t_prev_ = now_;                                                                     \
  } while (0)
#else
#define TSTAMP(i) \
  do {            \
  } while (0)
#endif

__global__ __launch_bounds__(256) void tr_layer_fwd_kernel(TrLayerArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  TrSmem& s = *reinterpret_cast<TrSmem*>(smem_raw);
  const int seq = blockIdx.x, T = a.T;
  const int tid = threadIdx.x, l = tid & 63, wave = tid >> 6;
  const int r0 = 16 * wave;                   // this wave's token rows
  const size_t grow0 = (size_t)seq * T;       // global row of token 0
  const int col = l & 15, rq = 4 * (l >> 4);  // accumulator column / first row of this lane
#ifdef MTA_TR_STAMPS
  unsigned long long t_prev_ = __builtin_amdgcn_s_memtime();
#endif

  // Every global LOAD of the block is issued before the stores it would otherwise queue behind: on gfx950 one
  // in-order vmcnt covers loads and stores, so a load issued after stores is waited for with those stores drained
  // (a bias load per output tile after the previous tile's stores was one store round trip each).
  uint4 pre[8];
  chunk_load(a, 0, pre);
  {
    // every small parameter load in flight at once, then into LDS
    float v[8];
    const bool lo = tid < 128;
    v[0] = lo ? a.g1[tid] : 0.f;
    v[1] = lo ? a.bo[tid] : 0.f;
    v[2] = lo ? a.g2[tid] : 0.f;
    v[3] = lo ? a.b2[tid] : 0.f;
    v[4] = a.bqkv[tid];
    v[5] = lo ? a.bqkv[256 + tid] : 0.f;
    v[6] = a.b1[tid];
    v[7] = a.b1[256 + tid];
    if (lo) {
      s.prm[P_G1 + tid] = v[0];
      s.prm[P_BO + tid] = v[1];
      s.prm[P_G2 + tid] = v[2];
      s.prm[P_B2 + tid] = v[3];
      s.prm[P_BQKV + 256 + tid] = v[5];
    }
    s.prm[P_BQKV + tid] = v[4];
    s.prm[P_B1 + tid] = v[6];
    s.prm[P_B1 + 256 + tid] = v[7];
  }
  float2 xrow[16];
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const int t = r0 + rr;
    xrow[rr] = t < T ? *reinterpret_cast<const float2*>(a.xs + (grow0 + t) * TD + 2 * l) : make_float2(0.f, 0.f);
  }
  // RoPE (cos, sin) of this lane's accumulator elements: rows r0 + rq + r, pair index (16 nt + col) % 32 / 2
  // = col / 2 (nt even) or 8 + col / 2 (nt odd): 8 values, loaded with the other up-front loads
  float2 rp[2][4];
#pragma unroll
  for (int hi = 0; hi < 2; ++hi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = r0 + rq + r;
      rp[hi][r] = reinterpret_cast<const float2*>(a.rope)[(size_t)(t < T ? t : 0) * (THD / 2) + 8 * hi + (col >> 1)];
    }
  uint32_t dseed = 0, dthr = 0;
  float dscale = 1.f;
  if (a.seed) {
    const uint64_t sd = *a.seed;
    dseed = (uint32_t)(sd ^ (sd >> 32));
    dthr = (uint32_t)(a.drop_p * 65536.f + 0.5f);
    dscale = 1.0f / (1.0f - a.drop_p);
  }
  __syncthreads();  // prm visible
  TSTAMP(0);

  // ---- RMSNorm1: wave w normalises its 16 rows (2 columns per lane) -> s.a (bf16), xn, r1 ----
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const int t = r0 + rr;
    const float2 v = xrow[rr];
    float q = v.x * v.x + v.y * v.y;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off, 64);
    const float rs = rsqrtf(q * (1.0f / TD) + a.eps);
    const float y0 = v.x * rs * s.prm[P_G1 + 2 * l], y1 = v.y * rs * s.prm[P_G1 + 2 * l + 1];
    __bf16 b0 = (__bf16)y0, b1v = (__bf16)y1;
    s.a[t * TLD + 2 * l] = b0;
    s.a[t * TLD + 2 * l + 1] = b1v;
    if (t < T) {
      a.xn[(grow0 + t) * TD + 2 * l] = b0;
      a.xn[(grow0 + t) * TD + 2 * l + 1] = b1v;
      if (l == 0) a.r1[grow0 + t] = rs;
    }
  }
  // weight chunk i goes into LDS buffer i & 1 as soon as its loads land, and chunk i + 1's loads are issued right
  // then -- before the phase's global stores, so waiting for them never drains those stores (in-order vmcnt)
  chunk_store(s.w[0], pre);
  chunk_load(a, 1, pre);
  __syncthreads();
  TSTAMP(1);

  // ---- QKV: chunks 0..2 (q, k, v), 128 output features each ----
  const float scale = 0.17677669529663687f;  // 1 / sqrt(32)
  for (int c = 0; c < 3; ++c) {
    const __bf16* w = s.w[c & 1];
    f32x4 accs[8];
    {
      bf16x8 af[4];
      afrags(s.a, TLD, r0, af);
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) accs[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      rowblock(af, w, accs);
    }
    // buffer (c + 1) & 1 held chunk c - 1: every wave finished it before the previous phase's barrier
    chunk_store(s.w[(c + 1) & 1], pre);
    chunk_load(a, c + 2, pre);
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const f32x4 acc = accs[nt];
      const int f = 16 * nt + col;  // feature within q / k / v
      const float bias = s.prm[P_BQKV + c * TD + f];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = r0 + rq + r;
        const __bf16 hb = (__bf16)(acc[r] + bias);  // the saved (unrotated) qkv value
        if (t < T) a.qkv[(grow0 + t) * 3 * TD + c * TD + f] = hb;
        float x = t < T ? (float)hb : 0.f;
        if (c < 2) {
          // RoPE on (2i, 2i+1) pairs = adjacent lanes; angle index i = (f % 32) / 2
          const float px = __shfl_xor(x, 1, 64);
          const float2 cs = rp[nt & 1][r];
          x = (f & 1) ? (px * cs.y + x * cs.x) : (x * cs.x - px * cs.y);
          if (c == 0) x *= scale;
          (c == 0 ? s.q : s.k)[t * TLD + f] = (__bf16)x;
        } else {
          s.vt[f * PLD2 + t] = (__bf16)x;
        }
      }
    }
    __syncthreads();
  }
  TSTAMP(2);
  // chunk 3 (Wo) is in s.w[1]; s.w[0] (Wv) is free: W1_0 goes in now and W2_0's loads are issued before the
  // attention / proj / norm stores
  chunk_store(s.w[0], pre);
  chunk_load(a, 5, pre);
  // the proj residual (x rows in the accumulator layout), loaded before the attention's stores
  f32x4 xres[8];
#pragma unroll
  for (int nt = 0; nt < 8; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = r0 + rq + r;
      xres[nt][r] = t < T ? a.xs[(grow0 + t) * TD + 16 * nt + col] : 0.f;
    }

  // ---- attention: wave w = query tile w, heads one after another; O -> s.a (xn is dead) ----
  for (int h = 0; h < 4; ++h) {
    f32x4 sc[4];
#pragma unroll
    for (int ki = 0; ki < 4; ++ki) {
      sc[ki] = mm16(s.q, TLD, r0, s.k, TLD, 16 * ki, THD * h, THD, f32x4{0.f, 0.f, 0.f, 0.f});
      if (16 * ki + col >= T) sc[ki] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    }
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
      if (col == 0) a.lse[((size_t)seq * 4 + h) * TROWS + r0 + rq + r] = m + __logf(sum);
    }
#pragma unroll
    for (int ki = 0; ki < 4; ++ki)
#pragma unroll
      for (int r = 0; r < 4; ++r) s.p[(r0 + rq + r) * PLD2 + 16 * ki + col] = (__bf16)sc[ki][r];
    // own P rows only: a wave reads back what it wrote (LDS ops of one wave complete in order)
#pragma unroll
    for (int dj = 0; dj < 2; ++dj) {
      const f32x4 ov = mm16(s.p, PLD2, r0, s.vt, PLD2, THD * h + 16 * dj, 0, TROWS, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = r0 + rq + r;
        const int f = THD * h + 16 * dj + col;
        const __bf16 ob = (__bf16)ov[r];
        s.a[t * TLD + f] = ob;
        if (t < T) a.o[(grow0 + t) * TD + f] = ob;
      }
    }
  }
  __syncthreads();
  TSTAMP(3);

  // ---- proj + residual: x1 = x + o Wo^T + bo (chunk 3 in s.w[1]); kept in registers for the FFN residual ----
  f32x4 x1v[8];
  {
    bf16x8 af[4];
    afrags(s.a, TLD, r0, af);
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) x1v[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    rowblock(af, s.w[1], x1v);
  }
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) {
    f32x4 acc = x1v[nt];
    const int f = 16 * nt + col;
    const float bias = s.prm[P_BO + f];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = r0 + rq + r;
      acc[r] = (acc[r] + bias) + xres[nt][r];
      if (t < T) a.x1[(grow0 + t) * TD + f] = acc[r];
    }
    x1v[nt] = acc;
  }
  // ---- RMSNorm2 on x1 rows held as (4 rows x 8 features) per lane: row sums over lanes of one 16-lane group ----
  {
    float q[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float acc = 0.f;
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) acc += x1v[nt][r] * x1v[nt][r];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) acc += __shfl_xor(acc, off, 64);
      q[r] = rsqrtf(acc * (1.0f / TD) + a.eps);
    }
    __syncthreads();  // every wave finished reading o (s.a) for its proj
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const int f = 16 * nt + col;
      const float gm = s.prm[P_G2 + f];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = r0 + rq + r;
        const __bf16 yb = (__bf16)(x1v[nt][r] * q[r] * gm);
        s.a[t * TLD + f] = yb;
        if (t < T) a.xn2[(grow0 + t) * TD + f] = yb;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = r0 + rq + r;
      if (col == 0 && t < T) a.r2[grow0 + t] = q[r];
    }
  }
  __syncthreads();
  TSTAMP(4);

  // ---- FFN in four 128-wide slices: u_c = dropout(GELU(xn2 W1_c^T + b1_c)) -> s.q; acc2 += u_c W2_c^T ----
  f32x4 acc2[8];
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) acc2[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int fc = 0; fc < 4; ++fc) {
    const int c1 = 4 + 2 * fc;  // W1_fc in s.w[0]; W2_fc in flight, into s.w[1] below
    f32x4 accs[8];
    {
      bf16x8 af[4];
      afrags(s.a, TLD, r0, af);
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) accs[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      rowblock(af, s.w[0], accs);
    }
    // s.w[1] held Wo / W2_{fc-1}: every wave finished it before the previous barrier
    chunk_store(s.w[1], pre);
    if (c1 + 2 < NCHUNKS) chunk_load(a, c1 + 2, pre);
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const f32x4 acc = accs[nt];
      const int j = 128 * fc + 16 * nt + col;  // hidden unit
      const float bias = s.prm[P_B1 + j];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = r0 + rq + r;
        const float v = acc[r] + bias;
        float g = mta_gelu(v);
        if (a.seed) {
          const uint32_t m = (uint32_t)(grow0 + t);
          const uint32_t hsh = tr_pair_hash(dseed, m >> 1, (uint32_t)j);
          const uint32_t u16 = (m & 1) ? (hsh >> 16) : (hsh & 0xFFFFu);
          g *= u16 >= dthr ? dscale : 0.f;
        }
        const __bf16 ub = (__bf16)g;
        s.q[t * TLD + 16 * nt + col] = ub;
        if (t < T) {
          a.pre1[(grow0 + t) * TFF + j] = (__bf16)v;
          a.u[(grow0 + t) * TFF + j] = ub;
        }
      }
    }
    __syncthreads();  // W2_fc visible; every wave done with W1_fc (s.w[0])
    // acc2 += u_fc W2_fc^T: u rows of this wave only (written by this wave above)
    {
      bf16x8 af[4];
      afrags(s.q, TLD, r0, af);
      rowblock(af, s.w[1], acc2);
    }
    if (c1 + 2 < NCHUNKS) {
      chunk_store(s.w[0], pre);
      chunk_load(a, c1 + 3, pre);
    }
    __syncthreads();  // W1_{fc+1} visible; every wave done with W2_fc and its u rows
  }
  TSTAMP(5);
  // ---- x2 = x1 + acc2 + b2 ----
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) {
    const int f = 16 * nt + col;
    const float bias = s.prm[P_B2 + f];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = r0 + rq + r;
      if (t < T) a.x2[(grow0 + t) * TD + f] = (acc2[nt][r] + bias) + x1v[nt][r];
    }
  }
  TSTAMP(6);
}

}  // namespace

extern "C" int mta_tr_layer_fwd(int nseq, int T, int d, int dff, int heads, const float* xs, const void* wqkv,
                                const void* wo, const void* w1, const void* w2, const float* g1, const float* bqkv,
                                const float* bo, const float* g2, const float* b1, const float* b2, float eps,
                                void* xn, void* qkv, void* o, void* xn2, void* pre1, void* u, float* x1, float* x2,
                                float* r1, float* r2, float* lse, const float* rope, const uint64_t* seed,
                                float drop_p, hipStream_t st) {
  if (d != TD || dff != TFF || heads != 4 || T < 1 || T > TROWS || !rope) return 1;
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&tr_layer_fwd_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)sizeof(TrSmem)) == hipSuccess;
  if (!attr) return 2;
  TrLayerArgs a;
  a.xs = xs;
  a.wqkv = static_cast<const __bf16*>(wqkv);
  a.wo = static_cast<const __bf16*>(wo);
  a.w1 = static_cast<const __bf16*>(w1);
  a.w2 = static_cast<const __bf16*>(w2);
  a.g1 = g1;
  a.bqkv = bqkv;
  a.bo = bo;
  a.g2 = g2;
  a.b1 = b1;
  a.b2 = b2;
  a.eps = eps;
  a.xn = static_cast<__bf16*>(xn);
  a.qkv = static_cast<__bf16*>(qkv);
  a.o = static_cast<__bf16*>(o);
  a.xn2 = static_cast<__bf16*>(xn2);
  a.pre1 = static_cast<__bf16*>(pre1);
  a.u = static_cast<__bf16*>(u);
  a.x1 = x1;
  a.x2 = x2;
  a.r1 = r1;
  a.r2 = r2;
  a.lse = lse;
  a.rope = rope;
  a.seed = seed;
  a.drop_p = drop_p;
  a.T = T;
  tr_layer_fwd_kernel<<<nseq, 256, sizeof(TrSmem), st>>>(a);
  return 0;
}
