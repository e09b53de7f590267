// Fused attention half of the transformer-encoder block forward (BASELINE.json north-star config 4: d = 128, 4 heads
// of 32, T <= 64 tokens per sequence), one launch per block:
//   xn = RMSNorm1(x) g1 -> qkv = xn Wqkv^T + bqkv -> RoPE(q) / sqrt(32), RoPE(k) -> softmax(q k^T, keys >= T masked) v
//   -> x1 = x + o Wo^T + bo
// The unfused chain was 4 launches (RMSNorm, QKV GEMM, attention, projection GEMM + residual; 4.8 + 8.6 + 7.0 + 8.6 us
// per block in the r4 trace).  One 512-thread workgroup owns one sequence (64 padded token rows) and keeps q, k, V^T,
// P and o in LDS; the weights stream from L2 straight into MFMA B-fragment registers (every wave owns distinct output
// columns: 48 of the 384 QKV features, 16 of the 128 projection features).  Attention: wave w runs head w / 2 for
// query tiles 2 (w % 2) and 2 (w % 2) + 1 (its own P rows: no barrier between scores and P V).
// Writes exactly what the unfused forward saves for the backward: xn, r1, qkv (UNROTATED, bias added, bf16), o, LSE,
// x1 -- staged through LDS into row-contiguous 16-B stores.
// Reference semantics: models/extras.py transformer_reference; ops/extras.py the unfused chain; csrc/attention.hip.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int AD = 128, AQ = 384, AHD = 32, AHEADS = 4, AT = 64, ATH = 512;
constexpr int BLD = AD + 8;   // bf16 [64][128] images
constexpr int QLD = AQ + 8;   // bf16 [64][384] staging
constexpr int VLD = AT + 8;   // bf16 [.][64] images (V^T, P)
constexpr int XLDF = AD + 4;  // fp32 [64][128] image

struct AttnFwdSmem {
  __bf16 xo[AT * BLD];          // xn (A of QKV), then o (A of the projection)
  __bf16 q[AT * BLD], k[AT * BLD];
  __bf16 vt[AD * VLD];
  union {
    __bf16 qkv[AT * QLD];       // qkv staging (copied out)
    __bf16 p[8][32 * VLD];      // per-wave P rows
    float x[AT * XLDF];         // x rows for the residual, then x1 staging
  } u;
  float2 rope[AT * (AHD / 2)];
  float g1[AD], bqkv[AQ], bo[AD];
};

struct AttnFwdArgs {
  const float* x;       // [M][128] block input (rows seq * T + t)
  const __bf16* wqkv;   // [384][128] fragment-major
  const __bf16* wo;     // [128][128] fragment-major
  const float *g1, *bqkv, *bo;
  const float* rope;    // [T][16] (cos, sin)
  float eps;
  int T;
  __bf16 *xn, *qkv, *o;
  float *r1, *lse, *x1;
  int split;  // 1: two workgroups per sequence, one per 32-query half (each recomputes the shared xn / k / v)
  int nfull;  // split == 0: workgroups below nfull own a whole sequence, the rest split the last sequences in halves
  // first block: the embedding x = in We^T + be computed here from the fp32 input tokens instead of read (in null:
  // x is read); x is then written to x_out (own rows) for the backward
  const float* in;   // [rows_in][F] (rows past rows_in: zero tokens, the padded sequences)
  const float* we;   // [128][F]
  const float* be;   // [128]
  int F, rows_in;
  float* x_out;
};

// B fragment from a fragment-major weight image (csrc/tr_ffn.hip frag_pack: 16 x 32 blocks of 1 KB, lane l's 8
// elements at l * 8): one wave's fragment is 1 KB contiguous instead of 16 rows x 64 B
__device__ __forceinline__ bf16x8 wfrag(const __bf16* w, int K, int n0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(w + ((size_t)((n0 >> 4) * (K >> 5) + (k0 >> 5)) << 9) + 8 * lane);
}
__device__ __forceinline__ bf16x8 lfrag(const __bf16* img, int ld, int r0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(img + (r0 + (lane & 15)) * ld + k0 + 8 * (lane >> 4));
}

__global__ __launch_bounds__(ATH) void tr_attn_fwd_kernel(AttnFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  AttnFwdSmem& s = *reinterpret_cast<AttnFwdSmem*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x, bs = a.split ? b : b - a.nfull;  // bs >= 0: a split workgroup, its index among them
  const bool split = bs >= 0;
  const int seq = split ? (a.split ? 0 : a.nfull) + (bs >> 1) : b, T = a.T;
  const int qh = split ? (bs & 1) : 0;  // query half (split): rows 32 qh .. 32 qh + 31 are this WG's
  auto own = [&](int r) { return !split || (r >> 5) == qh; };
  const size_t grow0 = (size_t)seq * T;
  const int rq = 4 * (lane >> 4), col = lane & 15;

  // ---- loads: QKV B fragments (this wave's 48 features x 4 k-steps), projection B fragments (16 features), x rows
  // (8 threads per row, 16 columns each), parameters and the RoPE table ----
  bf16x8 bq[4][3], bp[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) bq[ks][nt] = wfrag(a.wqkv, AD, 48 * wave + 16 * nt, 32 * ks, lane);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) bp[ks] = wfrag(a.wo, AD, 16 * wave, 32 * ks, lane);
  const int xr = tid >> 3, xc = 16 * (tid & 7);
  const bool rok = xr < T;
  float4 xv[4];
  if (a.in) {
    // embedding: 16 features x F inputs per thread (F = 3 for the financial windows)
    float tok[8];
    const size_t gr = grow0 + xr;
    const bool tin = rok && gr < (size_t)a.rows_in;
#pragma unroll
    for (int f = 0; f < 8; ++f) tok[f] = (f < a.F && tin) ? (float)(__bf16)a.in[gr * a.F + f] : 0.f;
    // this thread's 16 rows of We ([128][F] row-major: 16 F contiguous floats) and biases, as 16-B loads when F = 3
    // (the financial windows: 12 float4), scalar loads otherwise
    float wv[16 * 3], bv[16];
    const bool f3 = a.F == 3;
    if (f3) {
#pragma unroll
      for (int q4 = 0; q4 < 12; ++q4) {
        const float4 t4 = *reinterpret_cast<const float4*>(a.we + xc * 3 + 4 * q4);
        wv[4 * q4] = t4.x;
        wv[4 * q4 + 1] = t4.y;
        wv[4 * q4 + 2] = t4.z;
        wv[4 * q4 + 3] = t4.w;
      }
    }
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const float4 t4 = *reinterpret_cast<const float4*>(a.be + xc + 4 * q4);
      bv[4 * q4] = t4.x;
      bv[4 * q4 + 1] = t4.y;
      bv[4 * q4 + 2] = t4.z;
      bv[4 * q4 + 3] = t4.w;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float e[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int cc = 4 * i + kk, c = xc + cc;
        float v = bv[cc];
        // bf16 operands: the math of the unfused embedding GEMM
        if (f3) {
#pragma unroll
          for (int f = 0; f < 3; ++f) v = fmaf(tok[f], (float)(__bf16)wv[3 * cc + f], v);
        } else {
#pragma unroll
          for (int f = 0; f < 8; ++f)
            if (f < a.F) v = fmaf(tok[f], (float)(__bf16)a.we[c * a.F + f], v);
        }
        e[kk] = rok ? v : 0.f;
      }
      xv[i] = make_float4(e[0], e[1], e[2], e[3]);
      if (rok && own(xr)) *reinterpret_cast<float4*>(a.x_out + gr * AD + xc + 4 * i) = xv[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      xv[i] = rok ? *reinterpret_cast<const float4*>(a.x + (grow0 + xr) * AD + xc + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (tid < AD) {
    s.g1[tid] = a.g1[tid];
    s.bo[tid] = a.bo[tid];
  }
  if (tid < AQ) s.bqkv[tid] = a.bqkv[tid];
#pragma unroll
  for (int i = tid; i < AT * (AHD / 2); i += ATH) {
    const int t = i / (AHD / 2);
    s.rope[i] = t < T ? reinterpret_cast<const float2*>(a.rope)[i] : make_float2(1.f, 0.f);
  }
  __syncthreads();

  // ---- RMSNorm1 -> xn image, xn / r1 out ----
  {
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) q += xv[i].x * xv[i].x + xv[i].y * xv[i].y + xv[i].z * xv[i].z + xv[i].w * xv[i].w;
    q += __shfl_xor(q, 1, 64);
    q += __shfl_xor(q, 2, 64);
    q += __shfl_xor(q, 4, 64);
    const float rs = rsqrtf(q * (1.0f / AD) + a.eps);
    __bf16 yb[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float e[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) yb[4 * i + kk] = (__bf16)(e[kk] * rs * s.g1[xc + 4 * i + kk]);
    }
    uint4 p0, p1;
    __builtin_memcpy(&p0, yb, 16);
    __builtin_memcpy(&p1, yb + 8, 16);
    *reinterpret_cast<uint4*>(&s.xo[xr * BLD + xc]) = p0;
    *reinterpret_cast<uint4*>(&s.xo[xr * BLD + xc + 8]) = p1;
    if (rok && own(xr)) {
      *reinterpret_cast<uint4*>(a.xn + (grow0 + xr) * AD + xc) = p0;
      *reinterpret_cast<uint4*>(a.xn + (grow0 + xr) * AD + xc + 8) = p1;
      if ((tid & 7) == 0) a.r1[grow0 + xr] = rs;
    }
  }
  __syncthreads();

  // ---- QKV: 64 rows x this wave's 48 features, K = 128 ----
  f32x4 acc[4][3];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    bf16x8 af[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) af[mt] = lfrag(s.xo, BLD, 16 * mt, 32 * ks, lane);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) acc[mt][nt] = mfma16x16x32(af[mt], bq[ks][nt], acc[mt][nt]);
  }
  // bias -> bf16 qkv (saved unrotated); RoPE on q / k pairs (adjacent lanes), q scaled; V transposed
  const float scale = 0.17677669529663687f;  // 1 / sqrt(32)
#pragma unroll
  for (int nt = 0; nt < 3; ++nt) {
    const int c = 48 * wave + 16 * nt + col;  // feature in [0, 384)
    const int which = c >> 7, f = c & 127;     // q / k / v, feature within
    const float bias = s.bqkv[c];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * mt + rq + r;
        const __bf16 hb = (__bf16)(acc[mt][nt][r] + bias);
        s.u.qkv[t * QLD + c] = hb;
        float xval = (float)hb;
        if (which < 2) {
          const float px = __shfl_xor(xval, 1, 64);
          const float2 cs = s.rope[t * (AHD / 2) + ((f & (AHD - 1)) >> 1)];
          xval = (f & 1) ? (px * cs.y + xval * cs.x) : (xval * cs.x - px * cs.y);
          if (which == 0) xval *= scale;
          (which == 0 ? s.q : s.k)[t * BLD + f] = (__bf16)xval;
        } else {
          s.vt[f * VLD + t] = (__bf16)xval;
        }
      }
  }
  __syncthreads();  // qkv staging, q, k, V^T complete
  // qkv rows out (16-B pieces)
#pragma unroll
  for (int i = 0; i < AT * (AQ / 8) / ATH; ++i) {
    const int idx = tid + ATH * i, r = idx / (AQ / 8), c8 = idx % (AQ / 8);
    if (r < T && own(r))
      *reinterpret_cast<uint4*>(a.qkv + (grow0 + r) * AQ + 8 * c8) =
          *reinterpret_cast<const uint4*>(&s.u.qkv[r * QLD + 8 * c8]);
  }
  __syncthreads();  // staging read out before the P images reuse it

  // ---- attention: head h = wave / 2, query tiles 2 (wave & 1) + {0, 1} ----
  {
    const int h = wave >> 1;
    __bf16* pw = s.u.p[wave];  // this wave's 32 P rows
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      if (split && qq > 0) break;  // split: one query tile per wave (this half's tiles 2 qh, 2 qh + 1)
      const int qi = split ? 2 * qh + (wave & 1) : 2 * (wave & 1) + qq;
      f32x4 sc[4];
      const bf16x8 aq = lfrag(s.q, BLD, 16 * qi, AHD * h, lane);
#pragma unroll
      for (int ki = 0; ki < 4; ++ki) {
        sc[ki] = mfma16x16x32(aq, lfrag(s.k, BLD, 16 * ki, AHD * h, lane), f32x4{0.f, 0.f, 0.f, 0.f});
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
        if (col == 0) a.lse[((size_t)seq * AHEADS + h) * AT + 16 * qi + rq + r] = m + __logf(sum);
      }
#pragma unroll
      for (int ki = 0; ki < 4; ++ki)
#pragma unroll
        for (int r = 0; r < 4; ++r) pw[(16 * qq + rq + r) * VLD + 16 * ki + col] = (__bf16)sc[ki][r];
      // O tile (16 queries x 32 features of head h) = P (16 x 64) V (64 x 32): own P rows, written above
#pragma unroll
      for (int dj = 0; dj < 2; ++dj) {
        f32x4 ov = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          ov = mfma16x16x32(lfrag(pw, VLD, 16 * qq, 32 * kk, lane), lfrag(s.vt, VLD, AHD * h + 16 * dj, 32 * kk, lane),
                            ov);
#pragma unroll
        for (int r = 0; r < 4; ++r) s.xo[(16 * qi + rq + r) * BLD + AHD * h + 16 * dj + col] = (__bf16)ov[r];
      }
    }
  }
  __syncthreads();  // o image complete; P images dead
  // o rows out; x rows (residual) into the freed staging space
#pragma unroll
  for (int i = 0; i < AT * (AD / 8) / ATH; ++i) {
    const int idx = tid + ATH * i, r = idx / (AD / 8), c8 = idx % (AD / 8);
    if (r < T && own(r))
      *reinterpret_cast<uint4*>(a.o + (grow0 + r) * AD + 8 * c8) = *reinterpret_cast<const uint4*>(&s.xo[r * BLD + 8 * c8]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(&s.u.x[xr * XLDF + xc + 4 * i]) = xv[i];

  // ---- projection: x1 = x + o Wo^T + bo, this wave's 16 features x 64 rows ----
  f32x4 pacc[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                   f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      if (!split || (mt >> 1) == qh) pacc[mt] = mfma16x16x32(lfrag(s.xo, BLD, 16 * mt, 32 * ks, lane), bp[ks], pacc[mt]);
  __syncthreads();  // x rows staged
  {
    const int n = 16 * wave + col;
    const float bias = s.bo[n];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * mt + rq + r;
        s.u.x[t * XLDF + n] = (pacc[mt][r] + bias) + s.u.x[t * XLDF + n];
      }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < AT * (AD / 4) / ATH; ++i) {
    const int idx = tid + ATH * i, r = idx / (AD / 4), c4 = idx % (AD / 4);
    if (r < T && own(r))
      *reinterpret_cast<float4*>(a.x1 + (grow0 + r) * AD + 4 * c4) = *reinterpret_cast<const float4*>(&s.u.x[r * XLDF + 4 * c4]);
  }
}

// ---- backward tail of the attention half: d(xn) = dqkv Wqkv, then RMSNorm1 backward + residual ----
// dX = dX1 + rs (g1 o dxn - xhat mean(g1 o dxn o xhat)), xhat = x rs; dg1 += sum over rows of dxn o xhat.  The
// unfused chain was the input-gradient GEMM (6272 x 128 x 384, ~8.5 us) and the one-wave-per-row norm backward
// (~5.7 us).  One 512-thread workgroup per CU walking 32-row tiles, the next tile prefetched into registers: the dqkv tile, x and dX1 rows are staged
// through LDS by 16-B loads; wave w owns output features 16 w .. 16 w + 15 (Wqkv^T B fragments in registers from a
// fragment-major image, K = 384); the row statistic crosses the 8 waves once through LDS; dX leaves row-contiguous
// (fp32 and bf16); the dg1 partial row of each workgroup goes to a deferred norm slot (block-ordered sums).
constexpr int DXR = 32;         // rows per tile: 196 workgroups at the B=1 shape (64-row tiles: 98, 14.4 us)
constexpr int DQLD = AQ + 8;    // bf16 [32][384] dqkv tile
constexpr int XRLD = AD + 4;    // fp32 [32][128] rows
struct AttnDxSmem {
  __bf16 dq[DXR * DQLD];
  float x[DXR * XRLD];          // x rows, then dX rows (in place)
  float dr[DXR * XRLD];         // dX1 rows
  float red[8][DXR];            // per-wave row partials of sum(g1 dxn xhat)
  float rs[DXR];
};

struct AttnDxArgs {
  const __bf16* dqkv;   // [M][384]
  const __bf16* wqkvt;  // Wqkv^T fragment-major ([128][384])
  const float* x;       // [M][128] block input (RMSNorm1 input)
  const float* r1;      // [M] saved rstd
  const float* g1;      // [128]
  const float* dx1;     // [M][128] residual-stream gradient after the FFN half
  float* dx;            // [M][128] out, fp32
  __bf16* dxb;          // [M][128] out, bf16
  float* part;          // dg1 partial rows ([gridDim.x][part_ld])
  int part_ld;
  int M;
};

__global__ __launch_bounds__(ATH) void tr_attn_dx_kernel(AttnDxArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  AttnDxSmem& s = *reinterpret_cast<AttnDxSmem*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rq = 4 * (lane >> 4), col = lane & 15;
  const int c = 16 * wave + col;  // this lane's output feature
  bf16x8 bw[AQ / 32];
#pragma unroll
  for (int ks = 0; ks < AQ / 32; ++ks) bw[ks] = wfrag(a.wqkvt, AQ, 16 * wave, 32 * ks, lane);
  const float gc = a.g1[c];
  float dg = 0.f;  // this lane's share of dg1[c] (rows 4 (lane >> 4) + r of every tile)
  const int ntiles = (a.M + DXR - 1) / DXR;
  // a tile's operands are fetched into registers one tile ahead (its dqkv rows, x and dX1 rows, rstd) and written to
  // the LDS images at the tile's start: the loads of tile i + 1 fly under tile i's product and norm backward
  constexpr int NQ = DXR * (AQ / 8) / ATH, NX = DXR * (AD / 4) / ATH;
  uint4 pq[NQ];
  float4 px[NX], pd[NX];
  float prs = 0.f;
  auto fetch = [&](int tile) {
    const size_t row0 = (size_t)tile * DXR;
    const bool live = tile < ntiles;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int idx = tid + ATH * i, r = idx / (AQ / 8), c8 = idx % (AQ / 8);
      pq[i] = live && row0 + r < (size_t)a.M ? *reinterpret_cast<const uint4*>(a.dqkv + (row0 + r) * AQ + 8 * c8)
                                             : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int idx = tid + ATH * i, r = idx / (AD / 4), c4 = idx % (AD / 4);
      const bool ok = live && row0 + r < (size_t)a.M;
      px[i] = ok ? *reinterpret_cast<const float4*>(a.x + (row0 + r) * AD + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      pd[i] = ok ? *reinterpret_cast<const float4*>(a.dx1 + (row0 + r) * AD + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (tid < DXR) prs = live && row0 + tid < (size_t)a.M ? a.r1[row0 + tid] : 0.f;
  };
  fetch(blockIdx.x);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const size_t row0 = (size_t)tile * DXR;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int idx = tid + ATH * i, r = idx / (AQ / 8), c8 = idx % (AQ / 8);
      *reinterpret_cast<uint4*>(&s.dq[r * DQLD + 8 * c8]) = pq[i];
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int idx = tid + ATH * i, r = idx / (AD / 4), c4 = idx % (AD / 4);
      *reinterpret_cast<float4*>(&s.x[r * XRLD + 4 * c4]) = px[i];
      *reinterpret_cast<float4*>(&s.dr[r * XRLD + 4 * c4]) = pd[i];
    }
    if (tid < DXR) s.rs[tid] = prs;
    __syncthreads();
    fetch(tile + gridDim.x);
    // dxn tile: 32 rows x this wave's 16 features, K = 384
    constexpr int MT = DXR / 16;
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < AQ / 32; ++ks)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma16x16x32(lfrag(s.dq, DQLD, 16 * mt, 32 * ks, lane), bw[ks], acc[mt]);
    // g = g1 o dxn, xhat = x rs; per-row partial of sum(g xhat) over this wave's 16 features
    float gg[MT][4], xh[MT][4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * mt + rq + r;
        xh[mt][r] = s.x[t * XRLD + c] * s.rs[t];
        gg[mt][r] = acc[mt][r] * gc;
        dg = fmaf(acc[mt][r], xh[mt][r], dg);
        float p = gg[mt][r] * xh[mt][r];
        p += __shfl_xor(p, 1, 64);
        p += __shfl_xor(p, 2, 64);
        p += __shfl_xor(p, 4, 64);
        p += __shfl_xor(p, 8, 64);
        if (col == 0) s.red[wave][t] = p;
      }
    __syncthreads();  // red complete; every wave's reads of s.x done above
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * mt + rq + r;
        float s2 = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) s2 += s.red[w][t];
        s2 *= 1.0f / AD;
        s.x[t * XRLD + c] = s.rs[t] * (gg[mt][r] - xh[mt][r] * s2) + s.dr[t * XRLD + c];
      }
    __syncthreads();
    // dX rows out: fp32 and bf16, 16-B / 8-B pieces
#pragma unroll
    for (int i = 0; i < DXR * (AD / 4) / ATH; ++i) {
      const int idx = tid + ATH * i, r = idx / (AD / 4), c4 = idx % (AD / 4);
      if (row0 + r >= (size_t)a.M) continue;
      const float4 v = *reinterpret_cast<const float4*>(&s.x[r * XRLD + 4 * c4]);
      *reinterpret_cast<float4*>(a.dx + (row0 + r) * AD + 4 * c4) = v;
      bf16x4 b;
      b[0] = (__bf16)v.x;
      b[1] = (__bf16)v.y;
      b[2] = (__bf16)v.z;
      b[3] = (__bf16)v.w;
      *reinterpret_cast<bf16x4*>(a.dxb + (row0 + r) * AD + 4 * c4) = b;
    }
    __syncthreads();  // staging free for the next tile
  }
  // dg1 partial row of this workgroup: sum over the 4 row groups of each column, fixed order
  dg += __shfl_xor(dg, 16, 64);
  dg += __shfl_xor(dg, 32, 64);
  if (lane < 16) a.part[(size_t)blockIdx.x * a.part_ld + c] = dg;
}

}  // namespace

extern "C" int mta_tr_attn_fwd(int nseq, int T, int d, int heads, const float* x, const void* wqkv, const void* wo,
                               const float* g1, const float* bqkv, const float* bo, const float* rope, float eps,
                               void* xn, float* r1, void* qkv, void* o, float* lse, float* x1, const float* in,
                               const float* we, const float* be, int F, int rows_in, float* x_out, hipStream_t st) {
  if (d != AD || heads != AHEADS || T < 1 || T > AT || !rope) return 1;
  if (in && (F < 1 || F > 8 || !we || !be || !x_out)) return 3;
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&tr_attn_fwd_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)sizeof(AttnFwdSmem)) == hipSuccess;
  if (!attr) return 2;
  AttnFwdArgs a{};
  a.x = x;
  a.wqkv = static_cast<const __bf16*>(wqkv);
  a.wo = static_cast<const __bf16*>(wo);
  a.g1 = g1;
  a.bqkv = bqkv;
  a.bo = bo;
  a.rope = rope;
  a.eps = eps;
  a.T = T;
  a.xn = static_cast<__bf16*>(xn);
  a.qkv = static_cast<__bf16*>(qkv);
  a.o = static_cast<__bf16*>(o);
  a.r1 = r1;
  a.lse = lse;
  a.x1 = x1;
  a.in = in;
  a.we = we;
  a.be = be;
  a.F = F;
  a.rows_in = rows_in;
  a.x_out = x_out;
  // two workgroups per sequence (query halves): 2 x 104 sequences still fit one wave of workgroups on the 256 CUs,
  // and each recomputes only the shared norm / K / V (18.9 -> 16.7 us per launch, transformer B=1 0.576 -> 0.565 ms,
  // profiles/r4_bench_transformer_attn_split_ab.jsonl)
  // Beyond one wave of workgroups the duplicated norm / QKV work is pure cost (the 131 KB image allows one workgroup
  // per CU): transformer B=8 (800 sequences) ran 1,600 split workgroups at ~100 us per launch
  // (profiles/r6_transformer/tr_b8_kernel_stats.csv)
  a.split = (T > 32 && nseq <= 128) ? 1 : 0;
  // Above one wave of workgroups the last, partial wave splits its sequences in halves (the workgroups are
  // dispatched in index order, so those run last): transformer B=8, 832 sequences on 256 CUs, ends on 128 half
  // workgroups instead of 64 whole ones
  static const int n_cu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  const int rem = nseq % n_cu;
  a.nfull = (!a.split && T > 32 && nseq > n_cu && 2 * rem <= n_cu) ? nseq - rem : nseq;
  const int grid = a.split ? 2 * nseq : a.nfull + 2 * (nseq - a.nfull);
  tr_attn_fwd_kernel<<<grid, ATH, sizeof(AttnFwdSmem), st>>>(a);
  return 0;
}

// d(xn) = dqkv Wqkv and the RMSNorm1 backward with the residual gradient (see tr_attn_dx_kernel); dg1 into a deferred
// norm slot (mta_norm_flush sums it).  Returns non-zero on an unsupported shape.
extern "C" float* mta_norm_defer_slot(float* dgamma, float* dbeta, int D, int blocks, hipStream_t st, int* ld,
                                      long* pass);
extern "C" int mta_tr_attn_dx(int M, const void* dqkv, const void* wqkvt, const float* x, const float* r1,
                              const float* g1, const float* dx1, float* dx, void* dxb, float* dg1, hipStream_t st) {
  if (M < 1) return 1;
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&tr_attn_dx_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)sizeof(AttnDxSmem)) == hipSuccess;
  if (!attr) return 2;
  // one workgroup per CU is resident (~150 VGPRs at 8 waves: 2 waves per SIMD): a grid of exactly that walks the
  // tiles with the next tile's operands in flight (the old 1,024-workgroup grid ran B=8 as 4 rounds of 1-2 tiles)
  static const int n_cu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  const int tiles = (M + DXR - 1) / DXR;
  const int grid = tiles < n_cu ? tiles : n_cu;
  AttnDxArgs a{};
  int ld = 0;
  long pass = 0;
  a.part = mta_norm_defer_slot(dg1, nullptr, AD, grid, st, &ld, &pass);
  if (!a.part) return 3;
  a.dqkv = static_cast<const __bf16*>(dqkv);
  a.wqkvt = static_cast<const __bf16*>(wqkvt);
  a.x = x;
  a.r1 = r1;
  a.g1 = g1;
  a.dx1 = dx1;
  a.dx = dx;
  a.dxb = static_cast<__bf16*>(dxb);
  a.part_ld = ld;
  a.M = M;
  tr_attn_dx_kernel<<<grid, ATH, sizeof(AttnDxSmem), st>>>(a);
  return 0;
}
