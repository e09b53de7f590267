// Fused feed-forward half of the transformer-encoder block (BASELINE.json north-star config 4: d = 128, dff = 512),
// forward and input-gradient backward, one launch each (the weight gradients stay split-K GEMMs: they reduce over
// all M tokens).
//
// The unfused chain was 3 launches forward (RMSNorm2, FFN-up GEMM + GELU + dropout, FFN-down GEMM + residual) and
// 3 backward (two paired weight/input-gradient GEMMs, RMSNorm2 backward), each a ~6,000-row problem that is latency
// bound at 5-19 us per launch (r3 transformer trace).  Here one 512-thread workgroup owns 32 token rows (rows are
// independent in this half of the block), so M = 6,240 is 195 workgroups, and runs the whole chain with the
// activations in LDS:
//   forward : xn2 = RMSNorm(x1) g2 -> pre = xn2 W1^T + b1 -> u = dropout(GELU(pre)) -> x2 = x1 + u W2^T + b2
//   backward: du = dX W2 -> dpre = du * keep * gelu'(pre) -> dxn2 = dpre W1 -> dX1 = dX + RMSNorm2'(dxn2)
// Weight operands are streamed from L2 straight into MFMA B-fragment registers (16 B per lane, several k-steps in
// flight; every wave owns a distinct slice of the output columns, so nothing is shared across waves and no LDS
// round trip or barrier is needed for them).  Row activations are A fragments read from LDS images with 16-B
// padded rows (conflict-free ds_read_b128).  Global traffic is staged through LDS into row-contiguous 16-B stores.
// The backward takes the transposed bf16 weights (W2^T [512][128], W1^T [128][512], written by the forward's cast
// launch) so that both of its products are k-contiguous too.
// Dropout: the counter hash of the GEMM epilogues (gemm.hip gemm_pair_hash: pair of rows m >> 1, hidden unit j,
// 16-bit halves), so the fused and unfused paths draw identical masks.
// Reference semantics: models/extras.py transformer_reference (pre-norm block), ops/extras.py the unfused chain.
#include <algorithm>

#include "common.h"
#include "cast.h"

namespace {

#ifndef MTA_STAMPS
#define MTA_STAMPS 0
#endif
#if MTA_STAMPS
// probe build only (csrc/tools/ffn_probe.hip): s_memtime at the phase boundaries of every workgroup's wave 0
// ([direction][block][phase]), the per-phase split of one workgroup's critical path
__device__ unsigned long long mta_ffn_stamp[2][256][12];
#define FSTAMP(dir, k)                                                                                   \
  do {                                                                                                   \
    if ((threadIdx.x & 511) == 0 && blockIdx.x < 256) mta_ffn_stamp[(dir)][blockIdx.x][(k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// launch fill / drain in the globally consistent 100 MHz clock (the per-XCD shader clocks are not aligned)
#define FSTAMP_RT(dir, k)                                                                                \
  do {                                                                                                   \
    if ((threadIdx.x & 511) == 0 && blockIdx.x < 256) mta_ffn_stamp[(dir)][blockIdx.x][(k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define FSTAMP(dir, k) \
  do {                 \
  } while (0)
#define FSTAMP_RT(dir, k) \
  do {                    \
  } while (0)
#endif

constexpr int FD = 128, FF = 512, FBM = 32, FT = 512;  // 8 waves per 32-row workgroup
constexpr int XLD = FD + 8;    // bf16 row stride of [32][128] images (272 B)
constexpr int ULD = FF + 8;    // bf16 row stride of [32][512] images (1040 B)
constexpr int RLD = FD + 4;    // fp32 row stride of [32][128] row images (528 B)
constexpr int TLD = FBM + 8;   // bf16 row stride of transposed [features][32 tokens] images (80 B)

struct FfnFwdSmem {
  __bf16 xn[FBM * XLD];   // xn2 (A of FFN-up)
  __bf16 u[FBM * ULD];    // u   (A of FFN-down), then copied out
  __bf16 pre[FBM * ULD];  // pre-activation, copied out
  float x[FBM * RLD];     // x1 rows (residual), then x2 staging
  __bf16 uT[FF * TLD];    // u^T, xn2^T: the transposed (k-contiguous) weight-gradient operands
  __bf16 xnT[FD * TLD];
  float b1[FF], b2[FD], g2[FD];
};

struct FfnBwdSmem {
  __bf16 dx[FBM * XLD];    // dX (bf16, A of du = dX W2)
  __bf16 dpre[FBM * ULD];  // dpre (A of dxn2 = dpre W1), then copied out
  float x[FBM * RLD];      // x1 rows
  float g[FBM * RLD];      // dxn2 rows, then dX1 staging
  __bf16 dpreT[FF * TLD];  // dpre^T, dX^T: the transposed weight-gradient operands
  __bf16 dxT[FD * TLD];
  float g2[FD];
  float r[FBM];
};

struct FfnArgs {
  int M;
  float eps;
  const __bf16* w1;   // [512][128]  (backward: W1^T [128][512])
  const __bf16* w2;   // [128][512]  (backward: W2^T [512][128])
  const float *b1, *b2, *g2;
  const float* x1;    // [M][128] fp32
  const uint64_t* seed;
  float drop_p;
  // forward outputs
  __bf16 *xn2, *pre, *u;
  float *r2, *x2;
  // backward inputs / outputs
  const __bf16* dxb;  // dX as bf16 [M][128] (the weight-gradient operand already made by the previous launch)
  const float* dx;    // dX fp32 [M][128]
  const float* r2in;  // [M]
  const __bf16* prein;
  __bf16* dpre;       // [M][512]
  float* dx1;         // [M][128]
  __bf16* dx1b;       // [M][128]
  float* dg2;         // [128] += (f32 atomics, one per column and workgroup)
  // transposed weight-gradient operands [features][ldT] (token-contiguous; null: not written).  Forward: u^T, xn2^T;
  // backward: dpre^T, dX^T -- dW2 = dX^T u and dW1 = dpre^T xn2 then run as k-contiguous (NN) GEMMs
  __bf16 *uT, *xn2T, *dpreT, *dxT;
  int ldT;
};

// [features][32] transposed LDS image -> global [features][ldT] at token row0 (16-B pieces; M % 8 == 0)
template <int NF>
__device__ __forceinline__ void copy_out_t(const __bf16* img, __bf16* dst, int ldT, int row0, int M, int tid) {
#pragma unroll
  for (int i = 0; i < (NF * 4 + FT - 1) / FT; ++i) {
    const int idx = tid + FT * i, f = idx >> 2, c = idx & 3;
    if (f < NF && row0 + 8 * c < M)
      *reinterpret_cast<uint4*>(dst + (size_t)f * ldT + row0 + 8 * c) = *reinterpret_cast<const uint4*>(img + f * TLD + 8 * c);
  }
}

__device__ __forceinline__ uint32_t ffn_pair_hash(uint32_t s, uint32_t mpair, uint32_t n) {
  const uint32_t b = n * 0x85EBCA77u;  // == gemm.hip gemm_pair_hash
  uint32_t x = s ^ (mpair * 0x9E3779B1u) ^ ((b << 13) | (b >> 19));
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ bool ffn_keep(uint32_t dseed, uint32_t dthr, int m, int j) {
  const uint32_t h = ffn_pair_hash(dseed, (uint32_t)m >> 1, (uint32_t)j);
  const uint32_t u16 = (m & 1) ? (h >> 16) : (h & 0xFFFFu);
  return u16 >= dthr;
}

// B fragment of 16 output columns starting at n0, k-chunk k0 .. k0 + 31, from a k-contiguous [N][ldk] bf16 matrix
__device__ __forceinline__ bf16x8 bfrag(const __bf16* w, int ldk, int n0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(w + (size_t)(n0 + (lane & 15)) * ldk + k0 + 8 * (lane >> 4));
}
// The same fragment from a FRAGMENT-MAJOR image of a [N][K] matrix (frag_pack_kernel below): 16 x 32 blocks of 1 KB in
// (n / 16, k / 32) order, lane l's 8 elements at l * 8 -- one wave's fragment is 1 KB contiguous (8 full cache lines)
// instead of 16 rows x 64 B (16 half-used lines): the fused kernels' weight loads were ~14k of their ~34k cycles per
// workgroup (profiles/r4_ffn_probe_stamps.txt, EXP 1)
__device__ __forceinline__ bf16x8 bfrag_fm(const __bf16* w, int K, int n0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(w + ((size_t)((n0 >> 4) * (K >> 5) + (k0 >> 5)) << 9) + 8 * lane);
}
// A fragment of 16 rows starting at r0, k-chunk k0, from an LDS image with row stride ld
__device__ __forceinline__ bf16x8 afrag(const __bf16* img, int ld, int r0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(img + (r0 + (lane & 15)) * ld + k0 + 8 * (lane >> 4));
}

// [32][width] bf16 LDS image -> global rows row0 .. (16-B pieces, row-contiguous)
template <int WIDTH, int LD>
__device__ __forceinline__ void copy_out_bf16(const __bf16* img, __bf16* dst, int row0, int M, int tid) {
  constexpr int PER_ROW = WIDTH / 8;
#pragma unroll
  for (int i = 0; i < FBM * PER_ROW / FT; ++i) {
    const int idx = tid + FT * i, r = idx / PER_ROW, c = idx % PER_ROW;
    if (row0 + r < M)
      *reinterpret_cast<uint4*>(dst + (size_t)(row0 + r) * WIDTH + 8 * c) =
          *reinterpret_cast<const uint4*>(img + r * LD + 8 * c);
  }
}
// [32][128] fp32 LDS image -> global rows
__device__ __forceinline__ void copy_out_f32(const float* img, float* dst, int row0, int M, int tid) {
#pragma unroll
  for (int i = 0; i < FBM * 32 / FT; ++i) {
    const int idx = tid + FT * i, r = idx >> 5, c = idx & 31;
    if (row0 + r < M)
      *reinterpret_cast<float4*>(dst + (size_t)(row0 + r) * FD + 4 * c) =
          *reinterpret_cast<const float4*>(img + r * RLD + 4 * c);
  }
}

// Both kernels are persistent over 32-row tiles (grid = min(tiles, CUs); each workgroup walks tile, tile + grid, ...):
// the LDS images allow one 512-thread workgroup per CU, so a one-tile-per-workgroup grid ran B >= 4 windows as
// serial rounds of load -> compute -> copy out with nothing overlapping them (transformer B=8: 1,500 tiles, ~6
// rounds).  In the loop a tile's stores drain under the next tile's loads and products; the forward also prefetches
// the next tile's x1 rows and re-reads each weight-fragment set (L2-resident) for the next tile as soon as this
// tile's product has consumed it; the backward re-reads its weights with the tile's operands at the tile's start.
// Register budget: 2 waves per SIMD leave 256 per wave -- weight fragments held across tiles, or the backward's
// next-tile operands prefetched, spilled.  Every lane-dependent address is re-derived each tile from an opaque copy of
// the thread index (else the compiler hoists ~100 loop-invariant addresses out of the loop and spills them).
__global__ __launch_bounds__(FT) void tr_ffn_fwd_kernel(FfnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  FfnFwdSmem& s = *reinterpret_cast<FfnFwdSmem*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntiles = (a.M + FBM - 1) / FBM;
  FSTAMP_RT(0, 10);
  FSTAMP(0, 0);

  // ---- every load first (one in-order vmcnt covers loads and stores on gfx950) ----
  // FFN-up B fragments: this wave's 64 hidden units (4 tiles) x 4 k-steps
  bf16x8 bw[4][4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      bw[ks][nt] = bfrag_fm(a.w1, FD, 64 * wave + 16 * nt, 32 * ks, lane);
  // x1 rows: 16 threads per row, 8 columns each
  float4 xv[2];
  auto load_x = [&](int tile, int t) {
    const int r = tile * FBM + (t >> 4), xc = 8 * (t & 15);
    const bool ok = tile < ntiles && r < a.M;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      xv[i] = ok ? *reinterpret_cast<const float4*>(a.x1 + (size_t)r * FD + xc + 4 * i) : make_float4(1.f, 1.f, 1.f, 1.f);
  };
  load_x(blockIdx.x, tid);
  {
    const float v0 = a.b1[tid];
    const float v2 = tid < FD ? a.b2[tid] : 0.f, v3 = tid < FD ? a.g2[tid] : 0.f;
    s.b1[tid] = v0;
    if (tid < FD) {
      s.b2[tid] = v2;
      s.g2[tid] = v3;
    }
  }
  // FFN-down B fragments: this wave's 16 output features x 16 k-steps
  bf16x8 bd[16];
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) bd[ks] = bfrag_fm(a.w2, FF, 16 * wave, 32 * ks, lane);
  uint32_t dseed = 0, dthr = 0;
  float dscale = 1.f;
  if (a.seed) {
    const uint64_t sd = *a.seed;
    dseed = (uint32_t)(sd ^ (sd >> 32));
    dthr = (uint32_t)(a.drop_p * 65536.f + 0.5f);
    dscale = 1.0f / (1.0f - a.drop_p);
  }

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row0 = tile * FBM;
    // every lane-dependent address is re-derived from an opaque copy of the thread index each tile: left loop-
    // invariant, the compiler hoists ~100 of them (64-bit row offsets, LDS offsets, weight-fragment addresses) out
    // of the tile loop and spills them
    int tid_l = threadIdx.x;
    asm volatile("" : "+v"(tid_l));
    const int tid = tid_l, lane = tid & 63, wave = tid >> 6, xr = tid >> 4, xc = 8 * (tid & 15);
    const int rq = 4 * (lane >> 4), col = lane & 15;
    const bool rok = row0 + xr < a.M;
    __syncthreads();  // g2 / biases in LDS (first tile); the previous tile's x2 image copied out
    FSTAMP(0, 1);

    // ---- RMSNorm2 ----
    {
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) q += xv[i].x * xv[i].x + xv[i].y * xv[i].y + xv[i].z * xv[i].z + xv[i].w * xv[i].w;
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) q += __shfl_xor(q, off, 64);
      const float rs = rsqrtf(q * (1.0f / FD) + a.eps);
      __bf16 yb[8];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float e[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) yb[4 * i + k] = (__bf16)(e[k] * rs * s.g2[xc + 4 * i + k]);
        *reinterpret_cast<float4*>(&s.x[xr * RLD + xc + 4 * i]) = xv[i];
      }
      uint4 p0;
      __builtin_memcpy(&p0, yb, 16);
      *reinterpret_cast<uint4*>(&s.xn[xr * XLD + xc]) = p0;
      if (a.xn2T) {
#pragma unroll
        for (int k = 0; k < 8; ++k) s.xnT[(xc + k) * TLD + xr] = yb[k];
      }
      if (rok) {
        if (a.xn2) *reinterpret_cast<uint4*>(a.xn2 + (size_t)(row0 + xr) * FD + xc) = p0;
        if ((tid & 15) == 0) a.r2[row0 + xr] = rs;
      }
    }
    load_x(tile + gridDim.x, tid);  // the next tile's rows fly under this tile's products
    __syncthreads();           // xn2 image complete
    FSTAMP(0, 2);
    if (a.xn2T) copy_out_t<FD>(s.xnT, a.xn2T, a.ldT, row0, a.M, tid);

    // ---- FFN-up: 32 rows x this wave's 64 hidden units, K = 128 ----
    f32x4 acc[2][4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 a0 = afrag(s.xn, XLD, 0, 32 * ks, lane), a1 = afrag(s.xn, XLD, 16, 32 * ks, lane);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        acc[0][nt] = mfma16x16x32(a0, bw[ks][nt], acc[0][nt]);
        acc[1][nt] = mfma16x16x32(a1, bw[ks][nt], acc[1][nt]);
      }
    }
    // the next tile's FFN-up fragments (L2-resident; re-read unconditionally, a branch here made the compiler keep
    // both copies live) fly under this tile's epilogue and FFN-down
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bw[ks][nt] = bfrag_fm(a.w1, FD, 64 * wave + 16 * nt, 32 * ks, lane);
    FSTAMP(0, 3);
    // bias, GELU, dropout (one hash per pair of rows) -> u and pre images
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int j = 64 * wave + 16 * nt + col;
        const float bias = s.b1[j];
        uint32_t hp[2] = {0u, 0u};
        if (a.seed) {
          const uint32_t mp = (uint32_t)(row0 + 16 * mt + rq) >> 1;
          hp[0] = ffn_pair_hash(dseed, mp, (uint32_t)j);
          hp[1] = ffn_pair_hash(dseed, mp + 1, (uint32_t)j);
        }
        bf16x4 ut;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = 16 * mt + rq + r;
          const float v = acc[mt][nt][r] + bias;
          float g = mta_gelu(v);
          if (a.seed) {
            const uint32_t u16 = (r & 1) ? (hp[r >> 1] >> 16) : (hp[r >> 1] & 0xFFFFu);
            g *= u16 >= dthr ? dscale : 0.f;
          }
          s.pre[lr * ULD + j] = (__bf16)v;
          s.u[lr * ULD + j] = (__bf16)g;
          ut[r] = (__bf16)g;
        }
        // four consecutive token rows of hidden unit j: one 8-byte write of the transposed image
        if (a.uT) *reinterpret_cast<bf16x4*>(&s.uT[j * TLD + 16 * mt + rq]) = ut;
      }
    __syncthreads();  // u / pre complete
    FSTAMP(0, 4);
    copy_out_bf16<FF, ULD>(s.pre, a.pre, row0, a.M, tid);
    if (a.u) copy_out_bf16<FF, ULD>(s.u, a.u, row0, a.M, tid);
    if (a.uT) copy_out_t<FF>(s.uT, a.uT, a.ldT, row0, a.M, tid);

    FSTAMP(0, 5);
    // ---- FFN-down: 32 rows x this wave's 16 output features, K = 512 ----
    f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const bf16x8 a0 = afrag(s.u, ULD, 0, 32 * ks, lane), a1 = afrag(s.u, ULD, 16, 32 * ks, lane);
      o[0] = mfma16x16x32(a0, bd[ks], o[0]);
      o[1] = mfma16x16x32(a1, bd[ks], o[1]);
    }
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) bd[ks] = bfrag_fm(a.w2, FF, 16 * wave, 32 * ks, lane);
    FSTAMP(0, 6);
    // x2 = x1 + o + b2 into the x image (each wave its own 16 columns: no cross-wave hazard)
    {
      const int n = 16 * wave + col;
      const float bias = s.b2[n];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = 16 * mt + rq + r;
          s.x[lr * RLD + n] = (o[mt][r] + bias) + s.x[lr * RLD + n];
        }
    }
    __syncthreads();
    FSTAMP(0, 7);
    copy_out_f32(s.x, a.x2, row0, a.M, tid);
    FSTAMP(0, 8);
  }
  FSTAMP_RT(0, 11);
}

__global__ __launch_bounds__(FT) void tr_ffn_bwd_kernel(FfnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  FfnBwdSmem& s = *reinterpret_cast<FfnBwdSmem*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntiles = (a.M + FBM - 1) / FBM;
  FSTAMP_RT(1, 10);
  FSTAMP(1, 0);

  // ---- per tile, at its start: the weight fragments, dX (bf16) and the pre-activation tile for LDS, r2, x1 and dX
  // rows (fp32, 16 threads per row: first used at the tile's end) ----
  constexpr int PRE_PIECES = FBM * (FF / 8) / FT;
  uint4 dxp, prep[PRE_PIECES];
  float rp = 0.f;
  auto load_tile = [&](int tile, int tid) {  // the LDS operands of a tile: dX (bf16), the pre-activation tile, r2
    const int row0 = tile * FBM, xr = tid >> 4, xc = 8 * (tid & 15);
    const bool ok = row0 + xr < a.M;
    dxp = ok ? *reinterpret_cast<const uint4*>(a.dxb + (size_t)(row0 + xr) * FD + xc) : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int i = 0; i < PRE_PIECES; ++i) {
      const int idx = tid + FT * i, r = idx / (FF / 8), c = idx % (FF / 8);
      prep[i] = row0 + r < a.M ? *reinterpret_cast<const uint4*>(a.prein + (size_t)(row0 + r) * FF + 8 * c)
                               : make_uint4(0u, 0u, 0u, 0u);
    }
    if (tid < FBM) rp = row0 + tid < a.M ? a.r2in[row0 + tid] : 0.f;
  };
  if (tid < FD) s.g2[tid] = a.g2[tid];
  uint32_t dseed = 0, dthr = 0;
  float dscale = 1.f;
  if (a.seed) {
    const uint64_t sd = *a.seed;
    dseed = (uint32_t)(sd ^ (sd >> 32));
    dthr = (uint32_t)(a.drop_p * 65536.f + 0.5f);
    dscale = 1.0f / (1.0f - a.drop_p);
  }
  float dg2_acc = 0.f;  // this workgroup's dg2 column sums over its tiles (tid < FD), one atomic at the end

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row0 = tile * FBM;
    // every lane-dependent address is re-derived from an opaque copy of the thread index each tile: left loop-
    // invariant, the compiler hoists ~100 of them (64-bit row offsets, LDS offsets, weight-fragment addresses) out
    // of the tile loop and spills them
    int tid_l = threadIdx.x;
    asm volatile("" : "+v"(tid_l));
    const int tid = tid_l, lane = tid & 63, wave = tid >> 6, xr = tid >> 4, xc = 8 * (tid & 15);
    const int rq = 4 * (lane >> 4), col = lane & 15;
    const bool rok = row0 + xr < a.M;
    // du = dX W2 B fragments (W2^T [512][128]: this wave's 64 hidden units, 4 k-steps) and dxn2 = dpre W1 B fragments
    // (W1^T [128][512]: this wave's 16 features, 16 k-steps), re-read from L2 every tile with the tile's operands
    // (held across tiles, or re-read early, they spill: 2 waves per SIMD leave 256 registers)
    bf16x8 bw[4][4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bw[ks][nt] = bfrag_fm(a.w2, FD, 64 * wave + 16 * nt, 32 * ks, lane);
    load_tile(tile, tid);
    bf16x8 bd[16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) bd[ks] = bfrag_fm(a.w1, FF, 16 * wave, 32 * ks, lane);
    // this tile -> LDS (every reader of these images in the previous tile is behind its dxn2 barrier)
    *reinterpret_cast<uint4*>(&s.dx[xr * XLD + xc]) = dxp;
    if (a.dxT) {
      __bf16 e8[8];
      __builtin_memcpy(e8, &dxp, 16);
#pragma unroll
      for (int k = 0; k < 8; ++k) s.dxT[(xc + k) * TLD + xr] = e8[k];
    }
    // pre tile [32][512] -> the dpre image (the epilogue reads pre and writes dpre at the same element, same lane)
#pragma unroll
    for (int i = 0; i < PRE_PIECES; ++i) {
      const int idx = tid + FT * i, r = idx / (FF / 8), c = idx % (FF / 8);
      *reinterpret_cast<uint4*>(&s.dpre[r * ULD + 8 * c]) = prep[i];
    }
    if (tid < FBM) s.r[tid] = rp;
    float4 xt[2], gt[2];
    {
      const bool ok = row0 + xr < a.M;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        xt[i] = ok ? *reinterpret_cast<const float4*>(a.x1 + (size_t)(row0 + xr) * FD + xc + 4 * i)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
        gt[i] = ok ? *reinterpret_cast<const float4*>(a.dx + (size_t)(row0 + xr) * FD + xc + 4 * i)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    __syncthreads();  // dX image, pre tile, g2, r2
    FSTAMP(1, 1);

    // ---- du = dX W2: 32 rows x this wave's 64 hidden units, K = 128 ----
    f32x4 acc[2][4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 a0 = afrag(s.dx, XLD, 0, 32 * ks, lane), a1 = afrag(s.dx, XLD, 16, 32 * ks, lane);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        acc[0][nt] = mfma16x16x32(a0, bw[ks][nt], acc[0][nt]);
        acc[1][nt] = mfma16x16x32(a1, bw[ks][nt], acc[1][nt]);
      }
    }
    FSTAMP(1, 2);
    // dpre = du * keep / (1 - p) * gelu'(pre), in place over the pre tile
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int j = 64 * wave + 16 * nt + col;
        uint32_t hp[2] = {0u, 0u};
        if (a.seed) {
          const uint32_t mp = (uint32_t)(row0 + 16 * mt + rq) >> 1;
          hp[0] = ffn_pair_hash(dseed, mp, (uint32_t)j);
          hp[1] = ffn_pair_hash(dseed, mp + 1, (uint32_t)j);
        }
        bf16x4 dt;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = 16 * mt + rq + r;
          float v = acc[mt][nt][r];
          if (a.seed) {
            const uint32_t u16 = (r & 1) ? (hp[r >> 1] >> 16) : (hp[r >> 1] & 0xFFFFu);
            v *= u16 >= dthr ? dscale : 0.f;
          }
          v *= mta_gelu_grad((float)s.dpre[lr * ULD + j]);
          s.dpre[lr * ULD + j] = (__bf16)v;
          dt[r] = (__bf16)v;
        }
        if (a.dpreT) *reinterpret_cast<bf16x4*>(&s.dpreT[j * TLD + 16 * mt + rq]) = dt;
      }
    __syncthreads();  // dpre image complete
    FSTAMP(1, 3);
    if (a.dpre) copy_out_bf16<FF, ULD>(s.dpre, a.dpre, row0, a.M, tid);
    if (a.dpreT) copy_out_t<FF>(s.dpreT, a.dpreT, a.ldT, row0, a.M, tid);
    if (a.dxT) copy_out_t<FD>(s.dxT, a.dxT, a.ldT, row0, a.M, tid);

    FSTAMP(1, 4);
    // ---- dxn2 = dpre W1: 32 rows x this wave's 16 features, K = 512 ----
    f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const bf16x8 a0 = afrag(s.dpre, ULD, 0, 32 * ks, lane), a1 = afrag(s.dpre, ULD, 16, 32 * ks, lane);
      o[0] = mfma16x16x32(a0, bd[ks], o[0]);
      o[1] = mfma16x16x32(a1, bd[ks], o[1]);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) s.g[(16 * mt + rq + r) * RLD + 16 * wave + col] = o[mt][r];
    __syncthreads();  // dxn2 rows complete
    FSTAMP(1, 5);

    // ---- RMSNorm2 backward + residual, 16 threads per row:
    //   dx1 = dX + r (g2 dy) - x r^3 / d * sum(g2 dy x);  dg2 += dy x r ----
    {
      const float r = s.r[xr];
      float dyv[8], xe[8];
      float dot = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float4 dy4 = *reinterpret_cast<const float4*>(&s.g[xr * RLD + xc + 4 * i]);
        const float e[4] = {dy4.x, dy4.y, dy4.z, dy4.w};
        const float xx[4] = {xt[i].x, xt[i].y, xt[i].z, xt[i].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          dyv[4 * i + k] = e[k];
          xe[4 * i + k] = xx[k];
          dot = fmaf(s.g2[xc + 4 * i + k] * e[k], xx[k], dot);
        }
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) dot += __shfl_xor(dot, off, 64);
      const float c = dot * r * r * r * (1.0f / FD);
      float out[8];
      __bf16 ob[8];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float gd[4] = {gt[i].x, gt[i].y, gt[i].z, gt[i].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int e = 4 * i + k;
          out[e] = gd[k] + (r * s.g2[xc + e] * dyv[e] - xe[e] * c);
          ob[e] = (__bf16)out[e];
        }
      }
      __syncthreads();  // every row's dy read before the image is reused for dX1
#pragma unroll
      for (int i = 0; i < 2; ++i)
        *reinterpret_cast<float4*>(&s.g[xr * RLD + xc + 4 * i]) =
            make_float4(out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]);
      if (rok) {
        uint4 p0;
        __builtin_memcpy(&p0, ob, 16);
        *reinterpret_cast<uint4*>(a.dx1b + (size_t)(row0 + xr) * FD + xc) = p0;
      }
      // dg2: per-element dy x r into the x image (x is in registers), column sums after the barrier
#pragma unroll
      for (int i = 0; i < 2; ++i)
        *reinterpret_cast<float4*>(&s.x[xr * RLD + xc + 4 * i]) =
            make_float4(dyv[4 * i] * xe[4 * i] * r, dyv[4 * i + 1] * xe[4 * i + 1] * r,
                        dyv[4 * i + 2] * xe[4 * i + 2] * r, dyv[4 * i + 3] * xe[4 * i + 3] * r);
    }
    __syncthreads();
    FSTAMP(1, 6);
    copy_out_f32(s.g, a.dx1, row0, a.M, tid);
    if (tid < FD) {
      float cs = 0.f;
#pragma unroll 8
      for (int rr = 0; rr < FBM; ++rr) cs += s.x[rr * RLD + tid];
      dg2_acc += cs;
    }
    FSTAMP(1, 7);
  }
  if (tid < FD && blockIdx.x < ntiles) atomicAdd(a.dg2 + tid, dg2_acc);
  FSTAMP_RT(1, 11);
}

}  // namespace

extern "C" int mta_tr_ffn(int backward, int M, int d, int dff, float eps, const void* w1, const void* w2,
                          const float* b1, const float* b2, const float* g2, const float* x1, const uint64_t* seed,
                          float drop_p, void* xn2, void* pre, void* u, float* r2, float* x2, const void* dxb,
                          const float* dx, const float* r2in, const void* prein, void* dpre, float* dx1, void* dx1b,
                          float* dg2, void* uT, void* xn2T, void* dpreT, void* dxT, hipStream_t st) {
  if (d != FD || dff != FF || M < 1) return 1;
  if ((uT || xn2T || dpreT || dxT) && M % 8) return 3;
  FfnArgs a{};
  a.M = M;
  a.eps = eps;
  a.w1 = static_cast<const __bf16*>(w1);
  a.w2 = static_cast<const __bf16*>(w2);
  a.b1 = b1;
  a.b2 = b2;
  a.g2 = g2;
  a.x1 = x1;
  a.seed = seed;
  a.drop_p = drop_p;
  a.xn2 = static_cast<__bf16*>(xn2);
  a.pre = static_cast<__bf16*>(pre);
  a.u = static_cast<__bf16*>(u);
  a.r2 = r2;
  a.x2 = x2;
  a.dxb = static_cast<const __bf16*>(dxb);
  a.dx = dx;
  a.r2in = r2in;
  a.prein = static_cast<const __bf16*>(prein);
  a.dpre = static_cast<__bf16*>(dpre);
  a.dx1 = dx1;
  a.dx1b = static_cast<__bf16*>(dx1b);
  a.dg2 = dg2;
  a.uT = static_cast<__bf16*>(uT);
  a.xn2T = static_cast<__bf16*>(xn2T);
  a.dpreT = static_cast<__bf16*>(dpreT);
  a.dxT = static_cast<__bf16*>(dxT);
  a.ldT = M;
  // persistent: one workgroup per CU (the LDS images allow no more), each walking tiles blockIdx.x + k * grid
  static const int n_cu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  const int grid = std::min((M + FBM - 1) / FBM, n_cu);
  if (!backward) {
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&tr_ffn_fwd_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)sizeof(FfnFwdSmem)) == hipSuccess;
    if (!attr) return 2;
    tr_ffn_fwd_kernel<<<grid, FT, sizeof(FfnFwdSmem), st>>>(a);
  } else {
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&tr_ffn_bwd_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)sizeof(FfnBwdSmem)) == hipSuccess;
    if (!attr) return 2;
    tr_ffn_bwd_kernel<<<grid, FT, sizeof(FfnBwdSmem), st>>>(a);
  }
  return 0;
}

// ---- bf16 weight transposes for the backward (W1^T, W2^T of every layer in one launch) ----
namespace {
constexpr int WT_MAX = 32;
struct WtBatch {
  const __bf16* src[WT_MAX];
  __bf16* dst[WT_MAX];
  int rows[WT_MAX], cols[WT_MAX];
};
// dst[c][r] = src[r][c]; blockIdx.y = matrix, blockIdx.x = 64 x 64 tile
__global__ __launch_bounds__(256) void tr_wt_kernel(WtBatch b) {
  __shared__ __attribute__((aligned(16))) __bf16 t[64][72];
  const int mi = blockIdx.y, R = b.rows[mi], C = b.cols[mi];
  const int tiles_c = (C + 63) / 64;
  if ((int)blockIdx.x >= tiles_c * ((R + 63) / 64)) return;
  const int r0 = (blockIdx.x / tiles_c) * 64, c0 = (blockIdx.x % tiles_c) * 64;
  const __bf16* src = b.src[mi];
  __bf16* dst = b.dst[mi];
#pragma unroll
  for (int q = threadIdx.x; q < 512; q += 256) {
    const int r = q >> 3, ch = q & 7;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r0 + r < R && c0 + 8 * ch < C) v = *reinterpret_cast<const uint4*>(src + (size_t)(r0 + r) * C + c0 + 8 * ch);
    *reinterpret_cast<uint4*>(&t[r][8 * ch]) = v;
  }
  __syncthreads();
#pragma unroll
  for (int q = threadIdx.x; q < 512; q += 256) {
    const int c = q >> 3, ch = q & 7;
    if (c0 + c < C && r0 + 8 * ch < R) {
      __bf16 o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = t[8 * ch + i][c];
      uint4 v;
      __builtin_memcpy(&v, o, 16);
      *reinterpret_cast<uint4*>(dst + (size_t)(c0 + c) * R + r0 + 8 * ch) = v;
    }
  }
}
}  // namespace

// n matrices, src[i] bf16 [rows[i]][cols[i]] (rows, cols multiples of 8) -> dst[i] [cols[i]][rows[i]]
extern "C" int mta_tr_transpose_bf16(int n, const void* const* src, void* const* dst, const int* rows, const int* cols,
                                     hipStream_t st) {
  if (n < 1 || n > WT_MAX) return 1;
  WtBatch b{};
  int tiles = 1;
  for (int i = 0; i < n; ++i) {
    if (rows[i] % 8 || cols[i] % 8) return 2;
    b.src[i] = static_cast<const __bf16*>(src[i]);
    b.dst[i] = static_cast<__bf16*>(dst[i]);
    b.rows[i] = rows[i];
    b.cols[i] = cols[i];
    tiles = std::max(tiles, ((rows[i] + 63) / 64) * ((cols[i] + 63) / 64));
  }
  tr_wt_kernel<<<dim3(tiles, n), 256, 0, st>>>(b);
  return 0;
}

// ---- fp32 weights -> bf16 fragment-major [N][K] images (N % 16 == 0, K % 32 == 0), every one of a step in one
// launch: the fused FFN's W1, W2 (forward) and W2^T, W1^T (backward, tr: image(n, k) = src[k][n] of a [K][N] source),
// the fused attention half's W_qkv, W_o ----
namespace {
constexpr int FP_MAX = 32;
constexpr int FP_CAST_MAX = 4;
struct FragPackBatch {
  const float* src[FP_MAX];
  __bf16* dst[FP_MAX];
  int n[FP_MAX], k[FP_MAX], tr[FP_MAX];
  int count;
  // padded row-major casts riding along (the transformer's input tokens and embedding weight: the step's only other
  // cast work once the fused halves read fragment-major images) and the dropout seeds to advance: one launch
  CastItem cast[FP_CAST_MAX];
  int ncast;
  uint64_t* seeds;
  int nseeds;
};
__global__ __launch_bounds__(256) void frag_pack_kernel(FragPackBatch b) {
  if (blockIdx.x == 0 && blockIdx.y == 0 && (int)threadIdx.x < b.nseeds) b.seeds[threadIdx.x] += 0x9E3779B97F4A7C15ull;
  if ((int)blockIdx.y >= b.count) {
    cast_item_run(b.cast[blockIdx.y - b.count], blockIdx.x, gridDim.x);
    return;
  }
  const int mi = blockIdx.y, N = b.n[mi], K = b.k[mi];
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= N * K / 8) return;
  const int blk = c >> 6, lane = c & 63;
  const int n = 16 * (blk / (K >> 5)) + (lane & 15), k0 = 32 * (blk % (K >> 5)) + 8 * (lane >> 4);
  __bf16 e[8];
  if (!b.tr[mi]) {
    const float* s = b.src[mi] + (size_t)n * K + k0;
    const float4 x0 = *reinterpret_cast<const float4*>(s), x1 = *reinterpret_cast<const float4*>(s + 4);
    e[0] = (__bf16)x0.x; e[1] = (__bf16)x0.y; e[2] = (__bf16)x0.z; e[3] = (__bf16)x0.w;
    e[4] = (__bf16)x1.x; e[5] = (__bf16)x1.y; e[6] = (__bf16)x1.z; e[7] = (__bf16)x1.w;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = (__bf16)b.src[mi][(size_t)(k0 + i) * N + n];
  }
  uint4 v;
  __builtin_memcpy(&v, e, 16);
  *reinterpret_cast<uint4*>(b.dst[mi] + 8 * (size_t)c) = v;
}
}  // namespace

extern "C" int mta_frag_pack(int count, const float* const* src, void* const* dst, const int* n, const int* k,
                             const int* tr, int ncast, const float* const* csrc, void* const* cdst, const int* crows,
                             const int* ccols, const int* crows_p, const int* ccols_p, const int* cld,
                             uint64_t* seeds, int nseeds, hipStream_t st) {
  if (count < 1 || count > FP_MAX || ncast < 0 || ncast > FP_CAST_MAX || nseeds < 0 || nseeds > 256 ||
      (nseeds && !seeds))
    return 1;
  FragPackBatch b{};
  b.count = count;
  b.ncast = ncast;
  b.seeds = seeds;
  b.nseeds = nseeds;
  int chunks = 1;
  for (int i = 0; i < ncast; ++i) {
    b.cast[i] = CastItem{csrc[i], static_cast<__bf16*>(cdst[i]), crows[i], ccols[i], crows_p[i], ccols_p[i], cld[i]};
    const long e = (long)crows_p[i] * ccols_p[i] / ((ccols_p[i] & 7) == 0 ? 8 : 1);
    chunks = (int)std::max<long>(chunks, std::min<long>(e, 2048L * 256));
  }
  for (int i = 0; i < count; ++i) {
    if (n[i] < 16 || n[i] % 16 || k[i] < 32 || k[i] % 32) return 2;
    b.src[i] = src[i];
    b.dst[i] = static_cast<__bf16*>(dst[i]);
    b.n[i] = n[i];
    b.k[i] = k[i];
    b.tr[i] = tr[i];
    chunks = std::max(chunks, n[i] * k[i] / 8);
  }
  frag_pack_kernel<<<dim3((chunks + 255) / 256, count + ncast), 256, 0, st>>>(b);
  return 0;
}
