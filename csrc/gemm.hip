// bf16 MFMA GEMM for the MLP / transformer encoders (BASELINE.json north-star extras).
//
//   C[M,N] = alpha * sum_k A(m,k) * B(n,k)   (+ bias[n]) (GELU) (+ residual[m,n])
//
// A is stored row-major [M][K] (AT = false) or [K][M] (AT = true); B is stored [N][K] (BT = false,
// nn.Linear's weight layout) or [K][N] (BT = true).  The three products of a Linear layer map to:
//   forward   Y  = X  . W^T   A = X  [M][K],     B = W [N][K]          (AT=0, BT=0)
//   input grad dX = dY . W   A = dY [M][N],     B = W stored [N][K] = [k][n]  (AT=0, BT=1)
//   weight grad dW = dY^T . X A = dY stored [M][N] = [k][m], B = X stored [k][n] (AT=1, BT=1)
// so no transposed copies of weights or activations are ever materialised: the staging pass
// transposes 8x8 bf16 blocks in registers while writing the k-contiguous LDS images that make every
// MFMA fragment a single ds_read_b128.
//
// Tiles: BM x BN per 256-thread workgroup (4 waves in 2 x 2), BK = 32 (= one v_mfma_f32_16x16x32_bf16),
// register-staged prefetch of the next k-slice during the current slice's MFMAs, single LDS image with
// 80-byte rows (conflict-free b128 writes and reads).  Split-K (grid.z) accumulates with f32 atomics
// into an fp32 output (weight gradients straight into the flat gradient buffer); the weight-gradient
// form also produces the bias gradient (row sums of A over K) from the A fragments it already holds.
// Requirements (checked by the launcher): M, N, K multiples of 8, 16-byte aligned rows.
#include "common.h"

#include <algorithm>

extern "C" void mta_zero_bytes(void* dst, long bytes, hipStream_t st);  // optim.hip

namespace {

constexpr int GT = 256;  // threads per workgroup
constexpr int BK = 32;
constexpr int RS = 40;   // LDS row stride (bf16 elements): 32 + 8 pad = 80 B

// epilogue flags (applied in this order): BIAS, [aux_pre store], GELU, DROPOUT, DGELU, RESID
//   DGELU: v *= gelu'(aux_in[m][n]) (input-gradient GEMM of a GELU layer: dPre = dAct * gelu'(pre));
//   DROPOUT: v *= keep(seed, m, n) / (1 - p), the same hash the backward regenerates.
enum { EPI_BIAS = 1, EPI_GELU = 2, EPI_RESID = 4, EPI_ACCUM = 8, EPI_DROPOUT = 16, EPI_DGELU = 32 };

struct GemmArgs {
  const __bf16* A;
  const __bf16* B;
  int M, N, K, lda, ldb;
  float alpha;
  int flags;
  const float* bias;        // [N]
  const float* resid;       // [M][ldc] fp32 residual stream
  const __bf16* aux_in;     // [M][ldc] pre-activation for DGELU
  const uint64_t* seed;     // dropout seed (device scalar, advanced by the caller per step)
  float drop_p;
  __bf16* out_bf16;         // [M][ldc]
  float* out_f32;           // [M][ldc]  (EPI_ACCUM: +=, atomics when split-K)
  __bf16* aux_pre;          // [M][ldc]  pre-activation (GELU input) for the backward pass
  int ldc, n_store;        // columns [0, n_store) of C are written (N may include zero padding)
  int k_per_split;          // multiple of BK
  float* bias_grad;         // AT mode: += row sums of A over K  ([M])
  float* slab;              // split-K partials of the 256 x 256 kernel: [split][M][N] fp32 (null: f32 atomics)
  float* norm_parts;        // gradient producer: NORM_PARTS per-block sums of squares of the written output
  int overwrite;            // gradient producer: output = product (not += ), the optimizer left the range dirty
};
// per-block partials a gradient-producing GEMM writes for the fused optimizer's clip norm (optim.hip ext_parts)
constexpr int NORM_PARTS = 1024;


__device__ __forceinline__ uint4 and_mask(uint4 v, bool keep) {
  const uint32_t m = keep ? 0xFFFFFFFFu : 0u;  // bitwise AND: no select of aggregates (which goes via scratch)
  return make_uint4(v.x & m, v.y & m, v.z & m, v.w & m);
}

// GEMM-epilogue dropout (forward GELU epilogue and backward DGELU epilogue draw the same mask): one lowbias32 hash
// per PAIR of rows (a lane's 4 accumulator rows are 2 pairs), 16-bit uniform per element, p resolved to 1/65536:
// 2 multiplies per pair + 2 for the inputs instead of mta_hash3's 8 per element (the hash was ~30 us of the
// transformer step, r2 trace with / without dropout)
__device__ __forceinline__ uint32_t gemm_pair_hash(uint32_t s, uint32_t mpair, uint32_t n) {
  const uint32_t b = n * 0x85EBCA77u;
  uint32_t x = s ^ (mpair * 0x9E3779B1u) ^ ((b << 13) | (b >> 19));
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

union Bf8 {
  bf16x8 v;
  uint4 u;
  __bf16 e[8];
};

// GEMM epilogue store (nontemporal stores and store-less timing builds measured no gain: r3 probe, git history)
template <typename T>
__device__ __forceinline__ void epi_store(T* p, const T& v, int flags) {
  (void)flags;
  *p = v;
}

// Epilogue of one wave's MT x NT grid of 16x16 accumulator tiles whose top-left output element is (mbase, nbase):
// tile (i, j), register r of lane l holds C[mbase + 16 i + 4 (l >> 4) + r][nbase + 16 j + (l & 15)].  Rows are done
// IC tiles at a time; the operands the epilogue reads (residual stream, GELU input of a DGELU, the fp32 output of a
// non-split accumulate) are fetched for those IC x NT tiles first: interleaved with the output stores the compiler must
// keep each load behind the previous (possibly aliasing) store, i.e. one dependent global round trip per element (r2
// trace: 13 us per residual GEMM).
template <int MT, int NT, int IC>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, const f32x4 (&acc)[MT][NT], const int mbase,
                                              const int nbase, const bool split, const int lane) {
  const bool acc_rmw = (g.flags & EPI_ACCUM) && !split;  // read-modify-write of the fp32 output
  const bool prefetch = (g.flags & (EPI_RESID | EPI_DGELU)) || acc_rmw;
  uint32_t dseed = 0, dthr = 0;
  float dscale = 0.f;
  if (g.flags & EPI_DROPOUT) {
    const uint64_t sd = *g.seed;
    dseed = (uint32_t)(sd ^ (sd >> 32));
    dthr = (uint32_t)(g.drop_p * 65536.f + 0.5f);
    dscale = 1.0f / (1.0f - g.drop_p);
  }
#pragma unroll
  for (int i0 = 0; i0 < MT; i0 += IC) {
    float pre_in[IC][NT][4];
    if (prefetch) {
#pragma unroll
      for (int i = 0; i < IC; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int n = nbase + 16 * j + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = mbase + 16 * (i0 + i) + 4 * (lane >> 4) + r;
            const size_t o = (size_t)m * g.ldc + n;
            const bool ok = m < g.M && n < g.n_store;
            pre_in[i][j][r] = !ok ? 0.f : acc_rmw ? g.out_f32[o] : (g.flags & EPI_RESID) ? g.resid[o]
                                                                                         : (float)g.aux_in[o];
          }
        }
    }
#pragma unroll
    for (int i = 0; i < IC; ++i) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = nbase + 16 * j + (lane & 15);
        uint32_t hp[2] = {0u, 0u};
        if (g.flags & EPI_DROPOUT) {
          const uint32_t mp = (uint32_t)(mbase + 16 * (i0 + i) + 4 * (lane >> 4)) >> 1;
          hp[0] = gemm_pair_hash(dseed, mp, (uint32_t)n);
          hp[1] = gemm_pair_hash(dseed, mp + 1, (uint32_t)n);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mbase + 16 * (i0 + i) + 4 * (lane >> 4) + r;
          if (m >= g.M || n >= g.n_store) continue;
          float v = g.alpha * acc[i0 + i][j][r];
          const size_t o = (size_t)m * g.ldc + n;
          if (g.flags & EPI_ACCUM) {
            if (split) atomicAdd(g.out_f32 + o, v);
            else epi_store(g.out_f32 + o, pre_in[i][j][r] + v, g.flags);
            continue;
          }
          if (g.flags & EPI_BIAS) v += g.bias[n];
          if (g.aux_pre) epi_store(g.aux_pre + o, (__bf16)v, g.flags);
          if (g.flags & EPI_GELU) v = mta_gelu(v);
          if (g.flags & EPI_DROPOUT) {
            const uint32_t u16 = (r & 1) ? (hp[r >> 1] >> 16) : (hp[r >> 1] & 0xFFFFu);
            v *= u16 >= dthr ? dscale : 0.f;
          }
          if (g.flags & EPI_DGELU) v *= mta_gelu_grad(pre_in[i][j][r]);
          if (g.flags & EPI_RESID) v += pre_in[i][j][r];
          if (g.out_f32) epi_store(g.out_f32 + o, v, g.flags);
          if (g.out_bf16) epi_store(g.out_bf16 + o, (__bf16)v, g.flags);
        }
      }
    }
  }
}

template <int BM, int BN, int BKT, bool AT, bool BT>
__device__ __forceinline__ void gemm_body(const GemmArgs& g, const int bx, const int by, const int bz, const int gz,
                                          __bf16* __restrict__ As, __bf16* __restrict__ Bs) {
  constexpr int RST = BKT + 8;  // LDS row stride (bf16): BKT + 8 pad (16 B): conflict-free b128 rows
  constexpr int WM = BM / 2, WN = BN / 2, MT = WM / 16, NT = WN / 16;
  // staging work items: non-transposed = 16-B chunks (row, 8 k); transposed = 8x8 blocks (8 k-rows x 8 cols)
  constexpr int A_ITEMS = AT ? (BKT / 8) * (BM / 8) : BM * (BKT / 8);
  constexpr int B_ITEMS = BT ? (BKT / 8) * (BN / 8) : BN * (BKT / 8);
  constexpr int A_PER = (A_ITEMS + GT - 1) / GT;
  constexpr int B_PER = (B_ITEMS + GT - 1) / GT;
  constexpr int A_REGS = AT ? 8 : 1;  // 16-B loads per item
  constexpr int B_REGS = BT ? 8 : 1;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int n0 = bx * BN, m0 = by * BM;
  const int kbeg = bz * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  if (kbeg >= kend) return;

  typedef uint4 RegA[A_PER][A_REGS];
  typedef uint4 RegB[B_PER][B_REGS];
  RegA ra[1];
  RegB rb[1];
  uint32_t ma[1][A_PER], mb[1][B_PER];  // validity bits (one per 16-B load)

  // ---- global -> registers (raw values + masks; masks applied at LDS-store time) ----
  auto load = [&](RegA& ra, RegB& rb, uint32_t (&ma)[A_PER], uint32_t (&mb)[B_PER], int k0)
      __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < A_PER; ++p) {
      const int it = tid + p * GT;
      uint32_t msk = 0;
      if constexpr (!AT) {
        const int r = it / (BKT / 8), c = it % (BKT / 8);
        const int m = m0 + r, k = k0 + 8 * c;
        const bool ok = (it < A_ITEMS) & (m < g.M) & (k < kend);
        ra[p][0] = *reinterpret_cast<const uint4*>(g.A + (size_t)(ok ? m : 0) * g.lda + (ok ? k : 0));
        msk = ok ? 1u : 0u;
      } else {
        const int kb = it % (BKT / 8), mb8 = it / (BKT / 8);
        const int m = m0 + 8 * mb8;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int k = k0 + 8 * kb + i;
          const bool ok = (it < A_ITEMS) & (m < g.M) & (k < kend);
          ra[p][i] = *reinterpret_cast<const uint4*>(g.A + (size_t)(ok ? k : 0) * g.lda + (ok ? m : 0));
          msk |= ok ? 1u << i : 0u;
        }
      }
      ma[p] = msk;
    }
#pragma unroll
    for (int p = 0; p < B_PER; ++p) {
      const int it = tid + p * GT;
      uint32_t msk = 0;
      if constexpr (!BT) {
        const int r = it / (BKT / 8), c = it % (BKT / 8);
        const int n = n0 + r, k = k0 + 8 * c;
        const bool ok = (it < B_ITEMS) & (n < g.N) & (k < kend);
        rb[p][0] = *reinterpret_cast<const uint4*>(g.B + (size_t)(ok ? n : 0) * g.ldb + (ok ? k : 0));
        msk = ok ? 1u : 0u;
      } else {
        const int kb = it % (BKT / 8), nb8 = it / (BKT / 8);
        const int n = n0 + 8 * nb8;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int k = k0 + 8 * kb + i;
          const bool ok = (it < B_ITEMS) & (n < g.N) & (k < kend);
          rb[p][i] = *reinterpret_cast<const uint4*>(g.B + (size_t)(ok ? k : 0) * g.ldb + (ok ? n : 0));
          msk |= ok ? 1u << i : 0u;
        }
      }
      mb[p] = msk;
    }
  };

  // ---- registers -> LDS k-contiguous images (transposing 8x8 blocks for AT/BT) ----
  auto store = [&](const RegA& ra, const RegB& rb, const uint32_t (&ma)[A_PER], const uint32_t (&mb)[B_PER],
                   __bf16* __restrict__ As, __bf16* __restrict__ Bs) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < A_PER; ++p) {
      const int it = tid + p * GT;
      if (it >= A_ITEMS) continue;
      if constexpr (!AT) {
        const int r = it / (BKT / 8), c = it % (BKT / 8);
        *reinterpret_cast<uint4*>(&As[r * RST + 8 * c]) = and_mask(ra[p][0], ma[p] & 1u);
      } else {
        const int kb = it % (BKT / 8), mb8 = it / (BKT / 8);
        Bf8 in[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) in[i].u = and_mask(ra[p][i], (ma[p] >> i) & 1u);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          Bf8 o;
#pragma unroll
          for (int i = 0; i < 8; ++i) o.e[i] = in[i].e[j];
          *reinterpret_cast<uint4*>(&As[(8 * mb8 + j) * RST + 8 * kb]) = o.u;
        }
      }
    }
#pragma unroll
    for (int p = 0; p < B_PER; ++p) {
      const int it = tid + p * GT;
      if (it >= B_ITEMS) continue;
      if constexpr (!BT) {
        const int r = it / (BKT / 8), c = it % (BKT / 8);
        *reinterpret_cast<uint4*>(&Bs[r * RST + 8 * c]) = and_mask(rb[p][0], mb[p] & 1u);
      } else {
        const int kb = it % (BKT / 8), nb8 = it / (BKT / 8);
        Bf8 in[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) in[i].u = and_mask(rb[p][i], (mb[p] >> i) & 1u);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          Bf8 o;
#pragma unroll
          for (int i = 0; i < 8; ++i) o.e[i] = in[i].e[j];
          *reinterpret_cast<uint4*>(&Bs[(8 * nb8 + j) * RST + 8 * kb]) = o.u;
        }
      }
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rowsum[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) rowsum[i] = 0.f;
  const bool want_rowsum = g.bias_grad != nullptr && bx == 0 && wn == 0;

  auto compute = [&](const __bf16* __restrict__ As, const __bf16* __restrict__ Bs) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < BKT / 32; ++ks) {
      bf16x8 af[MT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        af[i] = *reinterpret_cast<const bf16x8*>(&As[(wm * WM + 16 * i + (lane & 15)) * RST + 32 * ks + 8 * (lane >> 4)]);
        if (want_rowsum) {
#pragma unroll
          for (int j = 0; j < 8; ++j) rowsum[i] += (float)af[i][j];
        }
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const bf16x8 bfr =
            *reinterpret_cast<const bf16x8*>(&Bs[(wn * WN + 16 * j + (lane & 15)) * RST + 32 * ks + 8 * (lane >> 4)]);
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i][j] = mfma16x16x32(af[i], bfr, acc[i][j]);
      }
    }
  };

  // single-stage loop: a two-stage form (two LDS images, loads two k-slices ahead) measured equal on mlp_large and
  // 0-10 % slower on the transformer's wgrad shapes (profiles/r4_gemm_pipe64_negative.txt) and was removed
  load(ra[0], rb[0], ma[0], mb[0], kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BKT) {
    __syncthreads();
    store(ra[0], rb[0], ma[0], mb[0], As, Bs);
    __syncthreads();
    if (k0 + BKT < kend) load(ra[0], rb[0], ma[0], mb[0], k0 + BKT);
    compute(As, Bs);
  }

  gemm_epilogue<MT, NT, MT>(g, acc, m0 + wm * WM, n0 + wn * WN, gz > 1, lane);
  if (want_rowsum) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float s = rowsum[i];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const int m = m0 + wm * WM + 16 * i + (lane & 15);
      if (lane < 16 && m < g.M) atomicAdd(g.bias_grad + m, s);
    }
  }
}

// XCD-aware block order: the dispatcher deals workgroup ids round-robin over the 8 XCDs (each with its own L2);
// remapping id -> (id % 8) * (nb / 8) + id / 8 gives every XCD a contiguous run of tiles (x fastest), so tiles that
// share A rows (and the same B column tiles) meet in one L2 instead of eight
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int nb8 = nb & ~7;
  return b < nb8 ? (b & 7) * (nb8 >> 3) + (b >> 3) : b;
}

template <int BM, int BN, int BKT>
constexpr int gemm_lds_elems() { return (BM + BN) * (BKT + 8); }

template <int BM, int BN, int BKT, bool AT, bool BT>
__global__ __launch_bounds__(GT) __attribute__((amdgpu_waves_per_eu(2))) void gemm_bf16_kernel(GemmArgs g, int nx, int ny, int nz) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[gemm_lds_elems<BM, BN, BKT>()];
  const int b = xcd_remap(blockIdx.x, nx * ny * nz);
  gemm_body<BM, BN, BKT, AT, BT>(g, b % nx, (b / nx) % ny, b / (nx * ny), nz, smem, smem + BM * (BKT + 8));
}

// ---- 256 x 256 macro-tile GEMM: LDS-DMA ring, staggered wave groups, in-kernel transposed operands ----
// The large problems (the mlp_large layers: 6400 x 2048 x 2048 and its two gradients) on one 512-thread workgroup per
// CU:
//   * 8 waves as 2 (M) x 4 (N); each wave owns 128 x 64 outputs = 8 x 4 accumulators of v_mfma_f32_16x16x32_bf16
//     (32 MFMAs per 32-deep k-tile against 12 fragment reads: the MFMA pipe, not LDS, is the limit);
//   * operands go global -> LDS by global_load_lds (16 B per lane, no VGPR round trip) into a ring of AHEAD + 2 k-tile
//     slots (A and B 16 KB each per slot; AHEAD = 3: 160 KB, the whole LDS), AHEAD k-tiles ahead of the one being
//     multiplied, waited with COUNTED vmcnt (never 0 in the loop) and raw s_barrier so the DMA stays in flight across
//     barriers (the latency to hide is an L2/MALL miss under full load, ~1-2 us);
//   * the two wave rows run one barrier apart ("ping-pong"): every k-tile is a [fragment reads + DMA issue] segment
//     and an [MFMA] segment separated by barriers, and the second wave row enters one barrier late, so on every
//     SIMD one wave multiplies while its partner reads -- s_setprio(1) around each MFMA cluster keeps the compiler
//     from moving MFMAs across the barriers;
//   * k-contiguous operands ([rows][K]) land as [256 rows][32 k] images (64-B rows) whose 16-B chunks are XOR-swizzled
//     by row bit 3 on the SOURCE address (the DMA writes lane-linear): conflict-free ds_read_b128 fragments;
//   * k-strided operands ([K][rows]: the input-gradient W and both weight-gradient operands) land untransposed as
//     [32 k][256 cols] images (512-B rows, 32-B chunks XOR-swizzled by k-row bits 0,1,3) and are read transposed by
//     ds_read_b64_tr_b16 (two per fragment), conflict-free: no transpose kernels, no transposing register staging.
// Ring hazards (j = k-tile; segments R = reads, M = DMA issue + MFMAs; row 0: R0 M0 R1 M1 ..., row 1: -- R0 M0 R1 ...):
//   WAR: tile j+AHEAD is issued during R_j into slot (j+AHEAD) % (AHEAD+2) = the slot of tile j-2; both rows retired
//        their reads of it (lgkmcnt(0) ahead of their MFMAs of M_{j-2}) before a barrier that precedes R_j;
//   RAW: row 0 first reads tile j+1 right after the barrier that closes its M_j, so at that barrier every wave has
//        waited for all but the tiles it issued after tile j+1 (row 0 at the end of M_j, row 1 at the end of R_j).
// Rows / columns beyond M, N are clamped on load (their outputs are not stored); K per split is a multiple of 32.
namespace big {
constexpr int TM = 256, TN = 256, KT = 32, THREADS = 512;
// DMA issued in the read segment, 3 k-tiles ahead, 5 slots (160 KB): r3 probe A/B against issuing it at the head of
// the MFMA segment (4 ahead, 5 slots): main loop 1832 -> 1555 cycles per k-tile, 4096^3 858 -> 892..1038 TF,
// mlp_large forward 545 -> 590 TF, input gradient 665 -> 707 TF (profiles/r3_gemm_variants.txt)
constexpr int AHEAD = 3;              // k-tiles in flight beyond the one multiplied
constexpr int SLOTS = AHEAD + 2;      // + the slot being read + the one whose reads retire during the issue
constexpr int OP_BYTES = 256 * KT * 2;     // one operand's k-tile image: 16 KB
constexpr int SLOT_BYTES = 2 * OP_BYTES;  // A | B
constexpr int EPI_ROW = 68;                                   // staged column: 64 f32 + 4 pad (epi_sidx)
constexpr int EPI_WAVE_BYTES = 64 * EPI_ROW * 4;               // 64 columns x 64 rows of one wave per pass
constexpr int LDS_BYTES = SLOTS * SLOT_BYTES > 8 * EPI_WAVE_BYTES ? SLOTS * SLOT_BYTES : 8 * EPI_WAVE_BYTES;

typedef short s16x4 __attribute__((ext_vector_type(4)));

// per-lane source of the two DMA instructions this wave issues for one operand of one k-tile
// (TW = image width in rows/columns; WAVES issuing)
template <bool T, int TW = 256, int WAVES = 8>
__device__ __forceinline__ void dma_src(const __bf16* base, int ld, int rows, int r0, int kbeg, int wave, int lane,
                                        const __bf16* (&src)[2]) {
  static_assert(TW / 16 == 2 * WAVES, "two 1-KB DMA pieces per wave and operand");
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int ins = wave + WAVES * q;  // 1-KB piece of the image
    if constexpr (!T) {
      // 16 rows x 64 B; lane -> (row, physical chunk); the chunk it holds is the swizzled logical one
      const int r = 16 * ins + (lane >> 2);
      const int c = (lane & 3) ^ (((r >> 3) & 1) << 1);
      const int row = min(r0 + r, rows - 1);
      src[q] = base + (size_t)row * ld + kbeg + 8 * c;
    } else {
      // 1024 / (2 TW) k-rows x 2 TW bytes; lane -> (k-row, 16-B unit); 32-B chunk swizzled by k-row
      constexpr int UPR = TW / 8;  // 16-B units per k-row
      const int kr = (1024 / (2 * TW)) * ins + lane / UPR, u = lane % UPR;
      const int h = (kr & 3) | (((kr >> 3) & 1) << 2);
      const int col = min(r0 + 16 * ((u >> 1) ^ h) + 8 * (u & 1), rows - 8);
      src[q] = base + (size_t)(kbeg + kr) * ld + col;
    }
  }
}

// diagnostic build (csrc/tools/gemm_probe.hip): s_memtime stamps of the main loop's segments, summed per wave
#ifdef MTA_STAMPS
__device__ unsigned long long stamp_acc[8][8];  // [wave][segment]
__device__ unsigned long long epi2_acc[8];       // GEMM_PROBE_EPI_TWICE: [wave] the second epilogue
#define GSTAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define GACC(i, a, b) dsum[i] += (unsigned)((b) - (a))
#else
#define GSTAMP(v)
#define GACC(i, a, b)
#endif

__device__ __forceinline__ void dma16(const __bf16* src, char* lds) {
  __builtin_amdgcn_global_load_lds(static_cast<const void*>(src), (lds_void*)(lds), 16, 0, 0);
}

// MFMA operand fragment of 16 rows (m or n) starting at image row/col `rb`, k-chunk lane >> 4
template <bool T, int TW = 256>
__device__ __forceinline__ bf16x8 frag(const char* img, int rb, int lane) {
  if constexpr (!T) {
    const int r = rb + (lane & 15);
    const int p = (lane >> 4) ^ (((lane >> 3) & 1) << 1);
    return *reinterpret_cast<const bf16x8*>(img + r * 64 + p * 16);
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int lc = rb >> 4;
    const int k0 = 8 * g + q, k1 = k0 + 4;
    const int h0 = (k0 & 3) | (((k0 >> 3) & 1) << 2), h1 = (k1 & 3) | (((k1 >> 3) & 1) << 2);
    // inline asm: the intrinsic form makes hipcc wait vmcnt(0) (every DMA in flight) before each transposed read;
    // the caller waits lgkmcnt(0) itself before the MFMAs (tr_wait)
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    u32x2 lo, hi;
    const unsigned a0 = (unsigned)(uintptr_t)(img + k0 * (2 * TW) + ((lc ^ h0) << 5) + 8 * p);
    const unsigned a1 = (unsigned)(uintptr_t)(img + k1 * (2 * TW) + ((lc ^ h1) << 5) + 8 * p);
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0) : "memory");
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a1) : "memory");
    const u32x2 v8[2] = {lo, hi};
    bf16x8 out;
    __builtin_memcpy(&out, v8, 16);
    return out;
  }
}

__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// outstanding DMA k-tiles this wave may leave in flight at a wait (immediate operand: one branch per count)
__device__ __forceinline__ void wait_tiles(int n) {
  if (n >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Epilogue through LDS (the ring is free once the loop's last barrier passed: every DMA and fragment read retired):
// each wave stages 64 of its 128 x 64 output rows at a time and reads them back row-contiguous, so
//   * plain outputs / operand reads are 16-B (f32) or 8-B (bf16) per lane, four full 256-B row segments per
//     instruction (the accumulator layout stores 4 rows x 64 B per instruction, 2-byte stores for bf16);
//   * split-K atomics are one 256-B row segment per instruction (lane = column).
// Its INSTRUCTION FOOTPRINT is what it costs: the instruction cache is cold when a tile gets there (every launch starts
// one), and every CU of the chip fetches the epilogue's lines one L2 round trip at a time.  The r5 stamp probe ran the
// same epilogue twice per tile: 68-94k cycles the first time, 30-43k the second (into a fresh buffer too: not a
// first-touch effect), against a ~100k-cycle main loop.  So the staging is column-major (ds_write_b128 of an
// accumulator's 4 rows: 16 writes per pass instead of 64 ds_write_b32 + selects), the read-back loops are ROLLED, and
// the common flag sets run a straight-line row loop specialised at compile time (rows_out_fast) instead of the
// general one's per-feature branches.  Staged element (col c, row r) of a wave's 64 x 64 pass sits at
// c * EPI_SP + (r ^ 4 ((c >> 2) & 7)): the b128 writes of 8 lanes (8 columns) and the ds_read2_b32 reads of a row's 4
// columns (c, c+1, c+2, c+3: dword offsets 0, 68, 136, 204) are both at most 2-way bank-conflicted.
// The reads are inline asm: hipcc would otherwise wait vmcnt(0) -- the previous iteration's stores -- ahead of every
// LDS access in a kernel that issues LDS-DMA.  `vec` = every pointer / ldc allows the wide forms.
constexpr int EPI_SP = 68;  // staged column pitch (floats)
__device__ __forceinline__ int epi_sidx(int c, int r) { return c * EPI_SP + (r ^ (((c >> 2) & 7) << 2)); }

typedef float f32x2 __attribute__((ext_vector_type(2)));
// staged row r, columns c0 .. c0 + 3 (c0 % 4 == 0), times alpha
__device__ __forceinline__ float4 stage_row4(const float* stage, int c0, int r, float alpha) {
  f32x2 lo, hi;
  const unsigned a = (unsigned)(uintptr_t)(stage + epi_sidx(c0, r));
  asm volatile("ds_read2_b32 %0, %2 offset1:68\n\tds_read2_b32 %1, %2 offset0:136 offset1:204\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(lo), "=v"(hi)
               : "v"(a)
               : "memory");
  return make_float4(lo.x * alpha, lo.y * alpha, hi.x * alpha, hi.y * alpha);
}
__device__ __forceinline__ float stage_one(const float* stage, int c, int r, float alpha) {
  float v;
  const unsigned a = (unsigned)(uintptr_t)(stage + epi_sidx(c, r));
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v * alpha;
}
// one pass's 4 x 4 accumulators (rows 16 ii + 4 (lane >> 4) + 0..3, column 16 j + (lane & 15)) into the stage
__device__ __forceinline__ void stage_pass(float* stage, const f32x4 (&acc)[8][4], const int i0, const int lane) {
#pragma unroll
  for (int ii = 0; ii < 4; ++ii)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned a = (unsigned)(uintptr_t)(stage + epi_sidx(16 * j + (lane & 15), 16 * ii + 4 * (lane >> 4)));
      asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(acc[i0 + ii][j]) : "memory");
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Straight-line row loop of the common flag sets (no accumulate, dropout, residual or GELU' operand; the wave's 128 x
// 64 block inside M x n_store; vec): F = EF_* bits, compile time
constexpr int EF_BIAS = 1, EF_GELU = 2, EF_F32 = 4, EF_BF16 = 8, EF_PRE = 16;
template <int F>
__device__ __forceinline__ void rows_out_fast(const GemmArgs& g, const float* stage, const int mrow, const int n,
                                              const int lane, const float (&bias4)[4]) {
  const int c0 = 4 * (lane & 15);
#pragma unroll 1
  for (int q = 0; q < 16; ++q) {
    const int rr = 4 * q + (lane >> 4);
    const float4 t = stage_row4(stage, c0, rr, g.alpha);
    const size_t o = (size_t)(mrow + rr) * g.ldc + n;
    float v[4] = {t.x, t.y, t.z, t.w};
    Bf8 pre;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (F & EF_BIAS) v[e] += bias4[e];
      if (F & EF_PRE) pre.e[e] = (__bf16)v[e];
      if (F & EF_GELU) v[e] = mta_gelu(v[e]);
    }
    if (F & EF_F32) *reinterpret_cast<float4*>(g.out_f32 + o) = make_float4(v[0], v[1], v[2], v[3]);
    if (F & EF_BF16) {
      Bf8 b;
#pragma unroll
      for (int e = 0; e < 4; ++e) b.e[e] = (__bf16)v[e];
      *reinterpret_cast<uint2*>(g.out_bf16 + o) = make_uint2(b.u.x, b.u.y);
    }
    if (F & EF_PRE) *reinterpret_cast<uint2*>(g.aux_pre + o) = make_uint2(pre.u.x, pre.u.y);
  }
}

// IN: the epilogue reads an operand per output (residual, GELU input of a DGELU, the fp32 output of a non-split
// accumulate).  The IN = false form has no global load in its loops: with loads on any path hipcc waits vmcnt(0) --
// every store issued so far -- ahead of the stores of each row (register reuse after a possibly outstanding load),
// one store round trip per row, which was ~40 % of a 256 x 256 tile's time (r4 epilogue probe).
template <bool IN>
__device__ __forceinline__ void big_rows_out(const GemmArgs& g, const float* stage, const int mrow, const int n,
                                          const int nc, const int lane, const bool vec, const bool split, const int bz,
                                          const float (&bias4)[4],
                                          const uint32_t dseed, const uint32_t dthr, const float dscale) {
  const bool accum = (g.flags & EPI_ACCUM) != 0;
  const int c0 = 4 * (lane & 15);
  if (accum && split && g.slab) {
    // split-K partial: plain 16-B stores into this split's slab; splitk_reduce_kernel adds the slabs afterwards
    float* slab = g.slab + (size_t)bz * g.M * g.N;
#pragma unroll 1
    for (int q = 0; q < 16; ++q) {
      const int rr = 4 * q + (lane >> 4);
      const float4 t = stage_row4(stage, c0, rr, g.alpha);
      if (mrow + rr < g.M && n + 3 < g.N) epi_store(reinterpret_cast<float4*>(slab + (size_t)(mrow + rr) * g.N + n), t, g.flags);
    }
    return;
  }
  if (accum && split) {  // nc: this lane's column of the 64-wide slice
#pragma unroll 1
    for (int rr = 0; rr < 64; ++rr) {
      const float v = stage_one(stage, lane, rr, g.alpha);
      if (mrow + rr < g.M && nc < g.n_store) atomicAdd(g.out_f32 + (size_t)(mrow + rr) * g.ldc + nc, v);
    }
    return;
  }
#pragma unroll 1
  for (int q = 0; q < 16; ++q) {
    const int rr = 4 * q + (lane >> 4);
    const int m = mrow + rr;
    const float4 t = stage_row4(stage, c0, rr, g.alpha);
    if (m >= g.M) continue;
    const size_t o = (size_t)m * g.ldc + n;
    const bool wide = vec && n + 3 < g.n_store;
    float pin[4] = {0.f, 0.f, 0.f, 0.f};
    if (IN) {
      if (wide) {
        if (accum || (g.flags & EPI_RESID)) {
          const float4 x = *reinterpret_cast<const float4*>((accum ? g.out_f32 : g.resid) + o);
          pin[0] = x.x; pin[1] = x.y; pin[2] = x.z; pin[3] = x.w;
        } else {
          Bf8 x;
          const uint2 u = *reinterpret_cast<const uint2*>(g.aux_in + o);
          x.u.x = u.x;
          x.u.y = u.y;
#pragma unroll
          for (int e = 0; e < 4; ++e) pin[e] = (float)x.e[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < g.n_store)
            pin[e] = accum ? g.out_f32[o + e] : (g.flags & EPI_RESID) ? g.resid[o + e] : (float)g.aux_in[o + e];
      }
    }
    float v[4] = {t.x, t.y, t.z, t.w};
    float pre[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (accum) {
        v[e] += pin[e];
        pre[e] = 0.f;
        continue;
      }
      v[e] += bias4[e];
      pre[e] = v[e];
      if (g.flags & EPI_GELU) v[e] = mta_gelu(v[e]);
      if (g.flags & EPI_DROPOUT) {
        const uint32_t h = gemm_pair_hash(dseed, (uint32_t)m >> 1, (uint32_t)(n + e));
        const uint32_t u16 = (m & 1) ? (h >> 16) : (h & 0xFFFFu);
        v[e] *= u16 >= dthr ? dscale : 0.f;
      }
      if (g.flags & EPI_DGELU) v[e] *= mta_gelu_grad(pin[e]);
      if (g.flags & EPI_RESID) v[e] += pin[e];
    }
    if (wide) {
      if (g.out_f32) epi_store(reinterpret_cast<float4*>(g.out_f32 + o), make_float4(v[0], v[1], v[2], v[3]), g.flags);
      if (!accum && g.out_bf16) {
        Bf8 b;
#pragma unroll
        for (int e = 0; e < 4; ++e) b.e[e] = (__bf16)v[e];
        epi_store(reinterpret_cast<uint2*>(g.out_bf16 + o), make_uint2(b.u.x, b.u.y), g.flags);
      }
      if (!accum && g.aux_pre) {
        Bf8 b;
#pragma unroll
        for (int e = 0; e < 4; ++e) b.e[e] = (__bf16)pre[e];
        epi_store(reinterpret_cast<uint2*>(g.aux_pre + o), make_uint2(b.u.x, b.u.y), g.flags);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (n + e >= g.n_store) continue;
        if (g.out_f32) g.out_f32[o + e] = v[e];
        if (!accum && g.out_bf16) g.out_bf16[o + e] = (__bf16)v[e];
        if (!accum && g.aux_pre) g.aux_pre[o + e] = (__bf16)pre[e];
      }
    }
  }
}

__device__ __forceinline__ void big_epilogue(const GemmArgs& g, const f32x4 (&acc)[8][4], const int mbase,
                                             const int nbase, const bool split, const int bz, const int lane,
                                             float* stage) {
  const bool accum = (g.flags & EPI_ACCUM) != 0;
  const bool vec = (g.ldc & 3) == 0 && ((uintptr_t)g.out_f32 & 15) == 0 && ((uintptr_t)g.out_bf16 & 7) == 0 &&
                   ((uintptr_t)g.aux_pre & 7) == 0 && ((uintptr_t)g.resid & 15) == 0 && ((uintptr_t)g.aux_in & 7) == 0;
  const int n = nbase + 4 * (lane & 15);  // this lane's 4 columns in the row-contiguous walk
  float bias4[4] = {0.f, 0.f, 0.f, 0.f};
  if (!accum && (g.flags & EPI_BIAS)) {
#pragma unroll
    for (int e = 0; e < 4; ++e) bias4[e] = n + e < g.N ? g.bias[n + e] : 0.f;
  }
  // the specialised form: its flag set, or -1
  int fast = -1;
  if (!accum && !(g.flags & (EPI_DROPOUT | EPI_DGELU | EPI_RESID)) && vec && mbase + 128 <= g.M &&
      nbase + 64 <= g.n_store)
    fast = ((g.flags & EPI_BIAS) ? EF_BIAS : 0) | ((g.flags & EPI_GELU) ? EF_GELU : 0) | (g.out_f32 ? EF_F32 : 0) |
           (g.out_bf16 ? EF_BF16 : 0) | (g.aux_pre ? EF_PRE : 0);
  uint32_t dseed = 0, dthr = 0;
  float dscale = 0.f;
  if (g.flags & EPI_DROPOUT) {
    const uint64_t sd = *g.seed;
    dseed = (uint32_t)(sd ^ (sd >> 32));
    dthr = (uint32_t)(g.drop_p * 65536.f + 0.5f);
    dscale = 1.0f / (1.0f - g.drop_p);
  }
  const bool in = (g.flags & (EPI_RESID | EPI_DGELU)) || (accum && !split);
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 0) stage_pass(stage, acc, 0, lane);
    else stage_pass(stage, acc, 4, lane);
    const int mrow = mbase + 64 * pass;
    switch (fast) {
      case EF_F32: rows_out_fast<EF_F32>(g, stage, mrow, n, lane, bias4); break;
      case EF_BIAS | EF_F32: rows_out_fast<EF_BIAS | EF_F32>(g, stage, mrow, n, lane, bias4); break;
      case EF_BIAS | EF_GELU | EF_F32 | EF_PRE:
        rows_out_fast<EF_BIAS | EF_GELU | EF_F32 | EF_PRE>(g, stage, mrow, n, lane, bias4);
        break;
      case EF_BF16: rows_out_fast<EF_BF16>(g, stage, mrow, n, lane, bias4); break;
      case EF_BIAS | EF_BF16: rows_out_fast<EF_BIAS | EF_BF16>(g, stage, mrow, n, lane, bias4); break;
      case EF_BIAS | EF_GELU | EF_BF16 | EF_PRE:
        rows_out_fast<EF_BIAS | EF_GELU | EF_BF16 | EF_PRE>(g, stage, mrow, n, lane, bias4);
        break;
      default: {
        const int nc = nbase + lane;
        if (in) big_rows_out<true>(g, stage, mrow, n, nc, lane, vec, split, bz, bias4, dseed, dthr, dscale);
        else big_rows_out<false>(g, stage, mrow, n, nc, lane, vec, split, bz, bias4, dseed, dthr, dscale);
      }
    }
    // the next pass re-stages over this one: every wave's reads above retired (inline-asm waits)
  }
}

// One (tile, k-range) segment's main loop: acc = A[m0 .. +256][kbeg .. kbeg + 32 nk) B[n0 .. +256][same k]^T for this
// wave's 128 x 64 slice; rowsum (want_rowsum) = row sums of this wave's A rows over the segment (bias gradients).
// Ends with both wave rows aligned at a barrier, every DMA retired: the ring is free for the epilogue's staging.
template <bool AT, bool BT>
__device__ __forceinline__ void mainloop(const GemmArgs& g, const int m0, const int n0, const int kbeg, const int nk,
                                         const bool want_rowsum, char* lds, f32x4 (&acc)[8][4], float (&rowsum)[8]) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const bool row1 = wm == 1;

  const __bf16* sa[2];
  const __bf16* sb[2];
  dma_src<AT>(g.A, g.lda, g.M, m0, kbeg, wave, lane, sa);
  dma_src<BT>(g.B, g.ldb, g.N, n0, kbeg, wave, lane, sb);
  const size_t stepA = AT ? (size_t)KT * g.lda : KT, stepB = BT ? (size_t)KT * g.ldb : KT;
  auto stage = [&](int j, int slot_i) __attribute__((always_inline)) {
    char* slot = lds + slot_i * SLOT_BYTES;
    const size_t oa = (size_t)j * stepA, ob = (size_t)j * stepB;
    dma16(sa[0] + oa, slot + wave * 1024);
    dma16(sa[1] + oa, slot + (wave + 8) * 1024);
    dma16(sb[0] + ob, slot + OP_BYTES + wave * 1024);
    dma16(sb[1] + ob, slot + OP_BYTES + (wave + 8) * 1024);
  };

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; ++i) rowsum[i] = 0.f;

  // prologue: k-tiles 0 .. AHEAD-1 into slots 0 .. AHEAD-1; tile 0 landed (every wave) at the first barrier
  const int pro = min(nk, AHEAD);
  for (int t = 0; t < pro; ++t) stage(t, t);
  wait_tiles(pro - 1);
  barrier();
  if (row1) barrier();  // the second wave row runs one barrier behind
  int rd = 0, wr = AHEAD % SLOTS;  // ring slots of tile j and of tile j + AHEAD
#ifdef MTA_STAMPS
  unsigned dsum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  GSTAMP(tloop0);
#endif
  for (int j = 0; j < nk; ++j) {
    GSTAMP(t0);
    // [reads] fragments of tile j
    const char* slot = lds + rd * SLOT_BYTES;
    bf16x8 af[8], bfr[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = frag<AT>(slot, wm * 128 + 16 * i, lane);
#pragma unroll
    for (int n = 0; n < 4; ++n) bfr[n] = frag<BT>(slot + OP_BYTES, wn * 64 + 16 * n, lane);
    if (j + AHEAD < nk) stage(j + AHEAD, wr);
    GSTAMP(t1);
    if (row1) wait_tiles(min(nk - 1, j + AHEAD) - (j + 1));
    GSTAMP(t2);
    barrier();
    GSTAMP(t3);
    // [MFMA] tile j (priority raised over the other wave row's reads: no-priority and static-priority builds
    // measured slower, profiles/r3_gemm_variants.txt)
    if (want_rowsum) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) rowsum[i] += (float)af[i][e];
    }
    if constexpr (AT || BT) {  // the transposed reads are inline asm: hipcc does not track them
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[i][n] = mfma16x16x32(af[i], bfr[n], acc[i][n]);
    __builtin_amdgcn_s_setprio(0);
    GSTAMP(t4);
    if (!row1) wait_tiles(min(nk - 1, j + AHEAD) - (j + 1));
    GSTAMP(t5);
    barrier();
    GSTAMP(t6);
    GACC(0, t0, t1);  // fragment reads (issue + completion: the stamp waits lgkmcnt)
    GACC(1, t1, t2);  // row 1: DMA wait
    GACC(2, t2, t3);  // barrier after the reads
    GACC(3, t3, t4);  // DMA issue + MFMA issue
    GACC(4, t4, t5);  // row 0: DMA wait
    GACC(5, t5, t6);  // barrier after the MFMAs
    rd = rd + 1 == SLOTS ? 0 : rd + 1;
    wr = wr + 1 == SLOTS ? 0 : wr + 1;
  }
  if (!row1) barrier();
#ifdef MTA_STAMPS
  GSTAMP(tloop1);
  GACC(6, tloop0, tloop1);
  if (lane == 0)
    for (int i = 0; i < 7; ++i) atomicAdd(&stamp_acc[wave][i], (unsigned long long)dsum[i]);
#endif
}

// bias gradient of the weight-gradient form: += this wave's row sums (f32 atomics, one per row and segment)
__device__ __forceinline__ void flush_rowsum(const GemmArgs& g, const float (&rowsum)[8], const int mrow0,
                                             const int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float s = rowsum[i];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const int m = mrow0 + 16 * i + (lane & 15);
    if (lane < 16 && m < g.M) atomicAdd(g.bias_grad + m, s);
  }
}

template <bool AT, bool BT>
__device__ __forceinline__ void body(const GemmArgs& g, int bx, int by, int bz, int gz, char* lds) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int m0 = by * TM, n0 = bx * TN;
  const int kbeg = bz * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = (kend - kbeg) / KT;
  if (nk <= 0) return;
  const bool want_rowsum = g.bias_grad != nullptr && bx == 0 && wn == 0;
  f32x4 acc[8][4];
  float rowsum[8];
  mainloop<AT, BT>(g, m0, n0, kbeg, nk, want_rowsum, lds, acc, rowsum);
#ifdef MTA_STAMPS
  GSTAMP(tepi0);
#endif
#ifdef GEMM_PROBE_EPI_SKIP  // probe build: no epilogue (the accumulators kept live), main loop + launch only
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
#else
  big_epilogue(g, acc, m0 + wm * 128, n0 + wn * 64, gz > 1, bz, lane,
               reinterpret_cast<float*>(lds + wave * EPI_WAVE_BYTES));
#endif
  if (want_rowsum) flush_rowsum(g, rowsum, m0 + wm * 128, lane);
#ifdef MTA_STAMPS
  GSTAMP(tend);
  if (lane == 0) atomicAdd(&stamp_acc[wave][7], (unsigned long long)(unsigned)(tend - tepi0));  // epilogue
#ifdef GEMM_PROBE_EPI_TWICE  // probe build: the same epilogue again, its code now in the instruction cache
  GemmArgs g2 = g;
#ifdef GEMM_PROBE_EPI_FRESH  // ... into a second output buffer (pages and lines not touched before)
  g2.out_f32 = g.out_f32 ? g.out_f32 + (size_t)g.M * g.ldc : nullptr;
  g2.aux_pre = g.aux_pre ? g.aux_pre + (size_t)g.M * g.ldc : nullptr;
#endif
  GSTAMP(t2a);
  big_epilogue(g2, acc, m0 + wm * 128, n0 + wn * 64, gz > 1, bz, lane,
               reinterpret_cast<float*>(lds + wave * EPI_WAVE_BYTES));
  GSTAMP(t2b);
  if (lane == 0) atomicAdd(&epi2_acc[wave], (unsigned long long)(unsigned)(t2b - t2a));
#endif
#endif
}

}  // namespace big


// out[m][n] (+)= sum over the splits of slab[z][m][n] (n < n_store), 4 columns per thread.  overwrite: out = sum (a
// gradient producer whose range the optimizer did not zero); norm_parts: every block's sum of squares of what it
// wrote (grid = NORM_PARTS blocks then), the clip norm's share of this range without another pass over it
__global__ __launch_bounds__(256) void splitk_reduce_kernel(float* __restrict__ out, int ldc, int n_store, int M, int N,
                                                            const float* __restrict__ slab, int splits, int overwrite,
                                                            float* __restrict__ norm_parts) {
  __shared__ float scratch[4];
  const int n4 = N >> 2;
  const long total = (long)M * n4;
  const size_t plane = (size_t)M * N;
  float sq = 0.f;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int m = (int)(e / n4), n = (int)(e - (long)m * n4) * 4;
    float4 s = *reinterpret_cast<const float4*>(slab + (size_t)m * N + n);
    for (int z = 1; z < splits; ++z) {
      const float4 t = *reinterpret_cast<const float4*>(slab + z * plane + (size_t)m * N + n);
      s.x += t.x;
      s.y += t.y;
      s.z += t.z;
      s.w += t.w;
    }
    float* o = out + (size_t)m * ldc + n;
    const float v[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (n + k < n_store) {
        const float r = overwrite ? v[k] : o[k] + v[k];
        o[k] = r;
        sq = fmaf(r, r, sq);
      }
  }
  if (norm_parts) {
    sq = block_sum(sq, scratch);
    if (threadIdx.x == 0) norm_parts[blockIdx.x] = sq;
  }
}

// norm partials of a contiguous fp32 range (gradient producers that did not take the slab path)
__global__ __launch_bounds__(256) void sumsq_parts_kernel(const float* __restrict__ x, long n, float* __restrict__ parts) {
  __shared__ float scratch[4];
  float sq = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    sq = fmaf(x[i], x[i], sq);
  sq = block_sum(sq, scratch);
  if (threadIdx.x == 0) parts[blockIdx.x] = sq;
}

template <bool AT, bool BT>
__global__ __launch_bounds__(big::THREADS) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_big_kernel(GemmArgs g, int nx, int ny, int nz) {
  extern __shared__ __attribute__((aligned(16))) char big_lds[];
  const int b = xcd_remap(blockIdx.x, nx * ny * nz);
  big::body<AT, BT>(g, b % nx, (b / nx) % ny, b / (nx * ny), nz, big_lds);
}

// Two independent GEMMs of one tile configuration in ONE launch (the backward's weight gradient and input
// gradient of a Linear read the same dY): one launch gap instead of two, and both grids fill the chip together.
// Blocks [0, n1) are problem 1 (x fastest, as a 3-D grid would be dispatched), [n1, n1 + n2) problem 2.
struct PairGrid {
  int nx1, ny1, nz1, nx2, ny2, nz2;
};
template <int BM, int BN, int BKT, bool AT1, bool BT1, bool AT2, bool BT2>
__global__ __launch_bounds__(GT) __attribute__((amdgpu_waves_per_eu(2))) void gemm_bf16_pair_kernel(GemmArgs g1, GemmArgs g2, PairGrid pg) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[gemm_lds_elems<BM, BN, BKT>()];
  __bf16* const As = smem;
  __bf16* const Bs = smem + BM * (BKT + 8);
  // XCD remap within each problem (a remap over the joint range deals the long weight-gradient tiles to the first
  // XCDs only: 295 -> 690 us per mlp_large pair); the second problem's ids stay on their XCD when n1 % 8 == 0
  const int n1 = pg.nx1 * pg.ny1 * pg.nz1;
  int b = blockIdx.x;
  b = b < n1 ? xcd_remap(b, n1) : ((n1 & 7) == 0 ? n1 + xcd_remap(b - n1, pg.nx2 * pg.ny2 * pg.nz2) : b);
  if (b < n1) {
    gemm_body<BM, BN, BKT, AT1, BT1>(g1, b % pg.nx1, (b / pg.nx1) % pg.ny1, b / (pg.nx1 * pg.ny1), pg.nz1, As,
                                           Bs);
  } else {
    b -= n1;
    gemm_body<BM, BN, BKT, AT2, BT2>(g2, b % pg.nx2, (b / pg.nx2) % pg.ny2, b / (pg.nx2 * pg.ny2), pg.nz2, As,
                                           Bs);
  }
}

// ---- grouped weight gradients ----
// The transformer backward's small weight gradients (out <= 512 x 512, K = 6,272 tokens) are latency-bound one by
// one: ~1 us per 128-deep k-step on a 64 x 64 tile, 8-12 us per launch at the best split
// (profiles/r4_wgrad_split_sweep.txt), ~180 us of the step.  Queued over the whole backward (defer = 2) and launched
// together (mta_gemm_group_flush: one launch per operand layout), their tiles x k-splits fill the chip with several
// workgroups per CU, whose k-step latencies then overlap instead of adding up.
constexpr int GROUP_MAX = 16;   // problems per launch (the table travels in the kernel arguments: < 4 KB)
// workgroup target of one grouped launch: 2 per CU.  The transformer B=1 set (17 problems, K = 6,272) on both launches:
// 74.8 us at 512, 80.6 at 1,024, 94.8 at 2,048, 108.5 at 256; 128 x 128 tiles 93-148 us (profiles/r5_wgrad_group_sweep.jsonl)
constexpr int GROUP_WGS = 512;
struct GroupTable {
  GemmArgs g[GROUP_MAX];
  int start[GROUP_MAX + 1];  // first block of each problem; start[n] = grid size
  int nx[GROUP_MAX], ny[GROUP_MAX], nz[GROUP_MAX];
  int n;
};
static_assert(sizeof(GroupTable) < 4000, "kernel arguments");
template <int BM, int BN, int BKT, bool T>  // T: both operands stored [K][rows] (dY^T X); else both k-contiguous
__global__ __launch_bounds__(GT) __attribute__((amdgpu_waves_per_eu(2))) void gemm_group_kernel(GroupTable t) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[gemm_lds_elems<BM, BN, BKT>()];
  int b = xcd_remap(blockIdx.x, t.start[t.n]);
  int p = 0;
  while (p + 1 < t.n && b >= t.start[p + 1]) ++p;
  b -= t.start[p];
  const int nx = t.nx[p], ny = t.ny[p];
  gemm_body<BM, BN, BKT, T, T>(t.g[p], b % nx, (b / nx) % ny, b / (nx * ny), t.nz[p], smem, smem + BM * (BKT + 8));
}

template <int BM, int BN, int BKT, bool AT, bool BT>
void launch(const GemmArgs& g, int ksplit, hipStream_t st) {
  const int nx = (g.N + BN - 1) / BN, ny = (g.M + BM - 1) / BM;
  const int blocks = nx * ny * ksplit;
  gemm_bf16_kernel<BM, BN, BKT, AT, BT><<<blocks, GT, 0, st>>>(g, nx, ny, ksplit);
}

// ---- big transposed-operand problems -> k-contiguous copies + the NN kernel ----
// The transposing register staging (8 loads per 8x8 block on half the threads, 64 byte moves per block) holds
// the input-gradient (B^T) and weight-gradient (A^T, B^T) GEMMs of mlp_large at 345 / 248 TFLOP/s against 460
// for the k-contiguous forward: above 2^31 MACs a 64x64-tile LDS transpose (~5.5 TB/s-class copy) into a
// per-operand workspace plus the NN kernel is cheaper.  Workspaces grow outside graph capture only and are never
// freed (a captured graph keeps pointing at the buffer it recorded); inside a capture that would need a larger one
// the GEMM keeps the transposing path.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const __bf16* __restrict__ in, int R, int C, int ld_in,
                                                             __bf16* __restrict__ out, int ld_out) {
  __shared__ __attribute__((aligned(16))) __bf16 t[64][72];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
#pragma unroll
  for (int q = threadIdx.x; q < 512; q += 256) {
    const int r = q >> 3, ch = q & 7;
    const int gr = r0 + r, gc = c0 + 8 * ch;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (gr < R && gc < C) v = *reinterpret_cast<const uint4*>(in + (size_t)gr * ld_in + gc);
    *reinterpret_cast<uint4*>(&t[r][8 * ch]) = v;
  }
  __syncthreads();
#pragma unroll
  for (int q = threadIdx.x; q < 512; q += 256) {
    const int c = q >> 3, ch = q & 7;  // output row c0 + c, input rows r0 + 8ch ... + 7
    const int oc = c0 + c, orow = r0 + 8 * ch;
    if (oc < C && orow < R) {
      Bf8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o.e[i] = t[8 * ch + i][c];
      *reinterpret_cast<uint4*>(out + (size_t)oc * ld_out + orow) = o.u;
    }
  }
}

// Per-(device, stream, slot) workspaces: 0 = weight-grad A^T, 1 = weight-grad B^T, 2 = input-grad B^T, 3 = split-K
// slabs of the 256 x 256 kernel.  Keyed by stream, so GEMMs issued eagerly on concurrent streams never share a
// buffer.  Grown outside graph capture only and never freed (a captured graph keeps pointing at the buffer it
// recorded); a capture stream borrows the smallest fitting buffer of its device (its eager warm-up's).
struct Workspace {
  int dev = -1;
  hipStream_t st = nullptr;
  int slot = -1;
  void* p = nullptr;
  size_t cap = 0;
};
Workspace g_ws[128];

__bf16* workspace(int slot, size_t bytes, hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  Workspace* w = nullptr;
  for (auto& e : g_ws)
    if (e.dev == dev && e.st == st && e.slot == slot) { w = &e; break; }
  if (w && bytes <= w->cap) return static_cast<__bf16*>(w->p);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    // no allocation inside a capture: a graph captured on its own stream (torch.cuda.graph) records the buffer its
    // eager warm-up used -- graph replays and eager steps are ordered on the one compute stream
    Workspace* best = nullptr;
    for (auto& e : g_ws)
      if (e.dev == dev && e.slot == slot && e.cap >= bytes && (!best || e.cap < best->cap)) best = &e;
    return best ? static_cast<__bf16*>(best->p) : nullptr;
  }
  if (!w) {
    for (auto& e : g_ws)
      if (e.dev < 0) { w = &e; break; }
    if (!w) return nullptr;
  }
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  w->dev = dev;
  w->st = st;
  w->slot = slot;
  w->p = p;  // the previous buffer is intentionally leaked (graphs may reference it)
  w->cap = bytes;
  return static_cast<__bf16*>(p);
}

// out[c][r] = in[r][c] for an R x C bf16 matrix (R, C multiples of 8)
void transpose(const __bf16* in, int R, int C, int ld_in, __bf16* out, hipStream_t st) {
  transpose_bf16_kernel<<<dim3((C + 63) / 64, (R + 63) / 64), 256, 0, st>>>(in, R, C, ld_in, out, R);
}

// rewrite a mode-1/2 problem as a mode-0 one over transposed copies; false = keep the transposing kernel
bool to_nn(GemmArgs& g, int mode, hipStream_t st) {
  if (mode == 0 || (long)g.M * g.N * g.K < (1L << 31)) return false;
  if (mode == 2) {
    __bf16* at = workspace(0, (size_t)g.M * g.K * sizeof(__bf16), st);
    __bf16* bt = workspace(1, (size_t)g.N * g.K * sizeof(__bf16), st);
    if (!at || !bt) return false;
    transpose(g.A, g.K, g.M, g.lda, at, st);  // A stored [K][M]
    transpose(g.B, g.K, g.N, g.ldb, bt, st);  // B stored [K][N]
    g.A = at;
    g.B = bt;
  } else {
    __bf16* bt = workspace(2, (size_t)g.N * g.K * sizeof(__bf16), st);
    if (!bt) return false;
    transpose(g.B, g.K, g.N, g.ldb, bt, st);  // B stored [K][N]
    g.B = bt;
  }
  g.lda = g.K;
  g.ldb = g.K;
  return true;
}

// tile configuration of a problem: 0 = 128x128x64, 1 = 128x128x32, 2 = 64x64x128, 3 = 64x64x32
inline int tile_config(const GemmArgs& g, int ksplit) {
  const long tiles128 = (long)((g.M + 127) / 128) * ((g.N + 127) / 128) * ksplit;
  const bool deep = g.k_per_split >= 128;
  return tiles128 >= 256 ? (deep ? 0 : 1) : (deep ? 2 : 3);
}

// pair kinds: 0 = two k-contiguous (NN) problems, 1 = (weight gradient, input gradient), 2 = two weight gradients
template <int BM, int BN, int BKT, int KIND>
void launch_pair_cfg(const GemmArgs& g1, int k1, const GemmArgs& g2, int k2, hipStream_t st) {
  PairGrid pg{(g1.N + BN - 1) / BN, (g1.M + BM - 1) / BM, k1, (g2.N + BN - 1) / BN, (g2.M + BM - 1) / BM, k2};
  const int blocks = pg.nx1 * pg.ny1 * pg.nz1 + pg.nx2 * pg.ny2 * pg.nz2;
  if constexpr (KIND == 0)
    gemm_bf16_pair_kernel<BM, BN, BKT, false, false, false, false><<<blocks, GT, 0, st>>>(g1, g2, pg);
  else if constexpr (KIND == 1)
    gemm_bf16_pair_kernel<BM, BN, BKT, true, true, false, true><<<blocks, GT, 0, st>>>(g1, g2, pg);
  else
    gemm_bf16_pair_kernel<BM, BN, BKT, true, true, true, true><<<blocks, GT, 0, st>>>(g1, g2, pg);
}

template <int KIND>
void launch_pair_kind(int c, const GemmArgs& g1, int k1, const GemmArgs& g2, int k2, hipStream_t st) {
  switch (c) {
    case 0: launch_pair_cfg<128, 128, 64, KIND>(g1, k1, g2, k2, st); break;
    case 1: launch_pair_cfg<128, 128, 32, KIND>(g1, k1, g2, k2, st); break;
    case 2: launch_pair_cfg<64, 64, 128, KIND>(g1, k1, g2, k2, st); break;
    default: launch_pair_cfg<64, 64, 32, KIND>(g1, k1, g2, k2, st); break;
  }
}

void dispatch_mode(int mode, const GemmArgs& g, int ksplit, hipStream_t st);

// ---- routing to the 256 x 256 kernel ----
// mta_gemm_set_big(0/1) turns it off / on at run time (tests compare the two paths in one process)
int g_big_override = -1;
inline bool big_on() { return g_big_override != 0; }

// split-K of the 256 x 256 kernel through fp32 slabs + one reduce launch (default) instead of fp32 atomics, which
// run at ~1 TB/s of added bytes chip-wide (mlp_large weight gradient: 64 MB of atomics = ~110k cycles per tile on
// the r3 stamp probe); MTA_GEMM_SLABS=0 keeps the atomics
inline bool slabs_on() {
  static const bool on = [] {
    const char* e = getenv("MTA_GEMM_SLABS");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <bool AT, bool BT>
void launch_big_t(const GemmArgs& g, int ksplit, hipStream_t st) {
  static const bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_big_kernel<AT, BT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, big::LDS_BYTES) == hipSuccess;
  }();
  (void)attr;
  const int nx = (g.N + big::TN - 1) / big::TN, ny = (g.M + big::TM - 1) / big::TM;
  GemmArgs ga = g;
  ga.slab = nullptr;
  if ((g.flags & EPI_ACCUM) && ksplit > 1 && slabs_on())
    ga.slab = reinterpret_cast<float*>(workspace(3, (size_t)ksplit * g.M * g.N * sizeof(float), st));
  gemm_big_kernel<AT, BT><<<nx * ny * ksplit, big::THREADS, big::LDS_BYTES, st>>>(ga, nx, ny, ksplit);
  if (ga.slab) {
    const long work = (long)g.M * (g.N / 4);
    const int blocks = g.norm_parts ? NORM_PARTS : (int)std::min<long>(4096, (work + 255) / 256);
    splitk_reduce_kernel<<<blocks, 256, 0, st>>>(g.out_f32, g.ldc, g.n_store, g.M, g.N, ga.slab, ksplit, g.overwrite,
                                                 g.norm_parts);
  }
}

// Eligible for the 256 x 256 kernel: 32-deep k-tiles and enough macro-tiles to fill at least half the CUs; the
// split-K accumulating form is re-split towards one wave of 256 workgroups (>= 8 k-tiles per split).  Returns the
// split it runs with (g.k_per_split updated), 0 = not eligible.
// workgroup target of the split accumulating form: one per CU (128 / 192 / 384 / 512 measured slower on mlp_large,
// profiles/r4_big_wgs_sweep.txt)
constexpr long BIG_WGS = 256;

int big_split(GemmArgs& g, int ksplit) {
  if (!big_on() || g.K % big::KT || g.M < 64 || g.N < 64) return 0;
  const long tiles = (long)((g.M + big::TM - 1) / big::TM) * ((g.N + big::TN - 1) / big::TN);
  if ((g.flags & EPI_ACCUM) && tiles * ksplit < BIG_WGS) {
    int ks = (int)std::max(1L, BIG_WGS / tiles);
    ks = std::min(ks, std::max(1, g.K / 256));
    if (ks > ksplit) {
      int kps = (g.K + ks - 1) / ks;
      kps = (kps + big::KT - 1) / big::KT * big::KT;
      ksplit = (g.K + kps - 1) / kps;
      g.k_per_split = kps;
    }
  }
  return tiles * ksplit < 128 ? 0 : ksplit;
}

bool big_eligible(const GemmArgs& g_in, int ksplit) {
  GemmArgs g = g_in;
  return big_split(g, ksplit) > 0;
}

bool try_big(int mode, const GemmArgs& g_in, int ksplit, hipStream_t st) {
  GemmArgs g = g_in;
  ksplit = big_split(g, ksplit);
  if (ksplit <= 0) return false;
  if (mode == 0) launch_big_t<false, false>(g, ksplit, st);
  else if (mode == 1) launch_big_t<false, true>(g, ksplit, st);
  else launch_big_t<true, true>(g, ksplit, st);
  return true;
}

// (weight-gradient, input-gradient) pair: modes (2, 1) with one tile configuration; false -> launch separately.
// Big pairs run on transposed copies (both NN) when both problems qualify.
bool launch_pair(const GemmArgs& g1_in, int k1, const GemmArgs& g2_in, int k2, hipStream_t st) {
  // big problems: the 256 x 256 kernel each (every one of them fills the chip on its own)
  if (big_eligible(g1_in, k1) && big_eligible(g2_in, k2)) {
    try_big(2, g1_in, k1, st);
    try_big(1, g2_in, k2, st);
    return true;
  }
  const int c = tile_config(g1_in, k1);
  if (c != tile_config(g2_in, k2)) return false;
  GemmArgs g1 = g1_in, g2 = g2_in;
  const bool nn1 = to_nn(g1, 2, st);
  const bool nn2 = nn1 && to_nn(g2, 1, st);
  if (nn1 && nn2) {
    launch_pair_kind<0>(c, g1, k1, g2, k2, st);
  } else if (nn1) {  // workspace for the second operand unavailable (capture): launch the two separately
    dispatch_mode(0, g1, k1, st);
    dispatch_mode(1, g2_in, k2, st);
  } else {
    launch_pair_kind<1>(c, g1, k1, g2, k2, st);
  }
  return true;
}

// two weight gradients (modes (2, 2), the transformer FFN's dW2 and dW1 after the fused input-gradient launch) in one
// launch when neither takes the 256 x 256 DMA kernel and both have one tile configuration
bool launch_pair_ww(const GemmArgs& g1, int k1, const GemmArgs& g2, int k2, hipStream_t st) {
  if (big_eligible(g1, k1) || big_eligible(g2, k2)) return false;
  if ((long)g1.M * g1.N * g1.K >= (1L << 31) || (long)g2.M * g2.N * g2.K >= (1L << 31)) return false;  // to_nn sizes
  const int c = tile_config(g1, k1);
  if (c != tile_config(g2, k2)) return false;
  launch_pair_kind<2>(c, g1, k1, g2, k2, st);
  return true;
}

// two accumulating products on k-contiguous operands (weight gradients from transposed activations, the transformer
// FFN's dW2 / dW1 with MTA_TR_WGRAD_NN=1) in one launch, same conditions as launch_pair_ww
bool launch_pair_nn_acc(const GemmArgs& g1, int k1, const GemmArgs& g2, int k2, hipStream_t st) {
  if (big_eligible(g1, k1) || big_eligible(g2, k2)) return false;
  const int c = tile_config(g1, k1);
  if (c != tile_config(g2, k2)) return false;
  launch_pair_kind<0>(c, g1, k1, g2, k2, st);
  return true;
}

template <bool AT, bool BT>
void dispatch(const GemmArgs& g, int ksplit, hipStream_t st) {
  // 128x128 tiles once they already fill the chip; 64x64 otherwise (these encoders' GEMMs are small).
  // K per workgroup >= 128: 128-deep k-steps (4 MFMA k-substeps per barrier pair) — the small-K GEMMs of the
  // transformer (K = 128) then stage once instead of paying four dependent load -> LDS -> MFMA rounds
  const long tiles128 = (long)((g.M + 127) / 128) * ((g.N + 127) / 128) * ksplit;
  const bool deep = g.k_per_split >= 128;
  // Per-CU balance of the k-contiguous deep case: 6400 x 2048 is 800 tiles of 128x128 = 3.125 per CU, so the
  // busiest CUs run 4 while the mean is 3.1 (78 %); 1,600 tiles of 128x64 = 6.25 per CU (89 %).  128x64 tiles cost
  // ~10 % per FLOP at equal balance (4096^3: 251 vs 226 us), so they are taken when 0.9 x their balance beats the
  // 128x128 balance: mlp_large forward 118 -> 108 us, step 1.69 -> 1.59 ms (profiles/r2_gemm_bn64_ab.txt).
  bool bn64 = false;
  if (deep && !AT && !BT) {
    constexpr long CUS = 256;
    const long t64 = (long)((g.M + 127) / 128) * ((g.N + 63) / 64) * ksplit;
    const double e128 = (double)tiles128 / (double)(CUS * ((tiles128 + CUS - 1) / CUS));
    const double e64 = (double)t64 / (double)(CUS * ((t64 + CUS - 1) / CUS));
    bn64 = 0.9 * e64 > e128;
  }
  if (tiles128 >= 256) {
    if (bn64) launch<128, 64, 64, AT, BT>(g, ksplit, st);
    else if (deep) launch<128, 128, 64, AT, BT>(g, ksplit, st);
    else launch<128, 128, 32, AT, BT>(g, ksplit, st);
  } else {
    if (deep) launch<64, 64, 128, AT, BT>(g, ksplit, st);
    else launch<64, 64, 32, AT, BT>(g, ksplit, st);
  }
}

void dispatch_mode(int mode, const GemmArgs& g_in, int ksplit, hipStream_t st) {
  if (try_big(mode, g_in, ksplit, st)) return;
  GemmArgs g = g_in;
  if (to_nn(g, mode, st)) mode = 0;
  if (mode == 0) dispatch<false, false>(g, ksplit, st);
  else if (mode == 1) dispatch<false, true>(g, ksplit, st);
  else dispatch<true, true>(g, ksplit, st);
}

// one deferred weight-gradient GEMM waiting for its input-gradient partner (stream-ordered, single-threaded use)
struct Pending {
  bool on = false;
  int mode = 2;  // 2: weight gradient dY^T X; 0: the same product on transposed (k-contiguous) operands
  GemmArgs g{};
  int ksplit;
  hipStream_t st;
} pending;

// weight gradients queued for one grouped launch per layout (kind 0: k-contiguous operands, 1: [K][rows] operands)
constexpr int GROUP_QMAX = 48;
constexpr long GROUP_SMALL_OUT = 512L * 512;  // outputs this small are always grouped (any K)
struct GroupQueue {
  GemmArgs g[2][GROUP_QMAX];
  int ks[2][GROUP_QMAX];  // requested split: 1 = none (deterministic mode), else chosen at the flush
  int n[2] = {0, 0};
  hipStream_t st = nullptr;
} gq;

// deep-K groups (every problem K >= GROUP_BIG_K: the transformer at B >= 4 windows) run on 128 x 128 tiles: at K =
// 48,000 (B=8) the 64 x 64 tiles' operand traffic per MFMA bound the two grouped launches (~360 us of a 1.94 ms step)
constexpr int GROUP_BIG_K = 16384;
#ifndef GROUP_BIG_TILES  // (diagnostic A/B builds: 0 keeps 64 x 64 tiles at any K)
#define GROUP_BIG_TILES 1
#endif
#ifndef GROUP_BIG_WGS  // workgroups a deep-K launch is sized to (2 resident per CU at 207 VGPRs; 256 / 1024 slower,
                       // profiles/r6_groupwgs/)
#define GROUP_BIG_WGS 512
#endif

void launch_group(int kind, int first, int count, hipStream_t st) {
  GroupTable t{};
  int kmin = 1 << 30;
  for (int q = first; q < first + count; ++q) kmin = std::min(kmin, gq.g[kind][q].K);
  const bool big = GROUP_BIG_TILES && kmin >= GROUP_BIG_K;
  const int TB = big ? 128 : 64;
  // one k-chunk for every problem of the launch, sized so that tiles x splits ~ GROUP_WGS
  long work = 0;
  for (int q = first; q < first + count; ++q) {
    const GemmArgs& g = gq.g[kind][q];
    work += (long)((g.M + TB - 1) / TB) * ((g.N + TB - 1) / TB) * g.K;
  }
  const long wgs = big ? GROUP_BIG_WGS : GROUP_WGS;
  long chunk = (work + wgs - 1) / wgs;
  chunk = std::max(256L, (chunk + 127) / 128 * 128);
  int blocks = 0;
  for (int q = 0; q < count; ++q) {
    GemmArgs g = gq.g[kind][first + q];
    int ks = gq.ks[kind][first + q] == 1 ? 1 : (int)std::max(1L, (g.K + chunk - 1) / chunk);
    int kps = (g.K + ks - 1) / ks;
    kps = (kps + BK - 1) / BK * BK;
    ks = (g.K + kps - 1) / kps;
    g.k_per_split = kps;
    t.g[q] = g;
    t.nx[q] = (g.N + TB - 1) / TB;
    t.ny[q] = (g.M + TB - 1) / TB;
    t.nz[q] = ks;
    t.start[q] = blocks;
    blocks += t.nx[q] * t.ny[q] * ks;
  }
  t.n = count;
  t.start[count] = blocks;
  if (big) {
    if (kind) gemm_group_kernel<128, 128, 64, true><<<blocks, GT, 0, st>>>(t);
    else gemm_group_kernel<128, 128, 64, false><<<blocks, GT, 0, st>>>(t);
  } else {
    if (kind) gemm_group_kernel<64, 64, 128, true><<<blocks, GT, 0, st>>>(t);
    else gemm_group_kernel<64, 64, 128, false><<<blocks, GT, 0, st>>>(t);
  }
}

}  // namespace

extern "C" void mta_gemm_set_big(int on) { g_big_override = on; }

// launch the queued weight gradients (end of a backward; also when the queue is full or the stream changes)
extern "C" void mta_gemm_group_flush() {
  for (int kind = 0; kind < 2; ++kind) {
    for (int first = 0; first < gq.n[kind]; first += GROUP_MAX)
      launch_group(kind, first, std::min(GROUP_MAX, gq.n[kind] - first), gq.st);
    gq.n[kind] = 0;
  }
}

// drop the queued weight gradients and a held-back GEMM unlaunched: their raw operand pointers are only kept alive by
// the caller of the backward that queued them (a backward that raised part-way must not leave them for the next flush)
extern "C" void mta_gemm_group_discard() {
  gq.n[0] = gq.n[1] = 0;
  pending.on = false;
}

// launch a deferred GEMM on its own (the caller's next GEMM was not its partner, or end of a backward)
extern "C" void mta_gemm_flush() {
  if (pending.on) {
    pending.on = false;
    dispatch_mode(pending.mode, pending.g, pending.ksplit, pending.st);
  }
}

namespace {

// gradient-producer request for the NEXT weight-gradient call (mta_gemm_grad_producer): overwrite its output range
// and / or write the clip-norm partials of it (the fused optimizer then neither zeroes nor re-reads that range)
struct ProducerReq {
  float* norm_parts = nullptr;
  bool overwrite = false;
} g_producer;

// whether dispatch_mode(2, g, ksplit) runs the 256 x 256 kernel with fp32 slabs (whose reduce launch overwrites and
// writes the partials itself)
bool slab_path(const GemmArgs& g_in, int ksplit, hipStream_t st) {
  if (!(g_in.flags & EPI_ACCUM) || !slabs_on()) return false;
  GemmArgs g = g_in;
  const int ks = big_split(g, ksplit);
  if (ks <= 1) return false;
  return workspace(3, (size_t)ks * g.M * g.N * sizeof(float), st) != nullptr;
}

// mode: 0 = NN-linear forward (AT=0,BT=0), 1 = input grad (AT=0,BT=1), 2 = weight grad (AT=1,BT=1)
int gemm_bf16_impl(int mode, const void* A, const void* B, int M, int N, int K, int lda, int ldb,
                   float alpha, int flags, const float* bias, const float* resid, const void* aux_in,
                   const uint64_t* seed, float drop_p, void* out_bf16, float* out_f32, void* aux_pre,
                   int ldc, int n_store, int ksplit, float* bias_grad, int defer, hipStream_t st) {
  if (n_store <= 0 || n_store > N) n_store = N;
  if (M % 8 || N % 8 || K % 8 || lda % 8 || ldb % 8 || ldc < n_store) return 1;
  if ((flags & EPI_ACCUM) == 0 && ksplit > 1) return 2;
  if ((flags & EPI_RESID) && (flags & EPI_DGELU)) return 7;  // one prefetched epilogue operand
  // bias gradient = row sums of A over K: the weight-gradient forms (mode 2, or mode 0 on transposed operands)
  if (bias_grad && !(mode == 2 || (mode == 0 && (flags & EPI_ACCUM)))) return 3;
  GemmArgs g{};
  g.A = static_cast<const __bf16*>(A);
  g.B = static_cast<const __bf16*>(B);
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = lda;
  g.ldb = ldb;
  g.alpha = alpha;
  g.flags = flags;
  g.bias = bias;
  g.resid = resid;
  g.aux_in = static_cast<const __bf16*>(aux_in);
  g.seed = seed;
  g.drop_p = drop_p;
  if ((flags & EPI_DROPOUT) && !seed) return 5;
  if ((flags & EPI_DGELU) && !aux_in) return 6;
  g.out_bf16 = static_cast<__bf16*>(out_bf16);
  g.out_f32 = out_f32;
  g.aux_pre = static_cast<__bf16*>(aux_pre);
  g.ldc = ldc;
  g.n_store = n_store;
  if (ksplit < 1) ksplit = 1;
  int kps = (K + ksplit - 1) / ksplit;
  kps = (kps + BK - 1) / BK * BK;
  ksplit = (K + kps - 1) / kps;
  g.k_per_split = kps;
  g.bias_grad = bias_grad;
  if (mode < 0 || mode > 2) return 4;
  const ProducerReq req = g_producer;
  g_producer = ProducerReq{};
  if (req.norm_parts || req.overwrite) {
    if (mode != 2 || defer || ldc != n_store || !(flags & EPI_ACCUM)) return 10;
    mta_gemm_flush();
    if (slab_path(g, ksplit, st)) {
      g.norm_parts = req.norm_parts;
      g.overwrite = req.overwrite ? 1 : 0;
      dispatch_mode(2, g, ksplit, st);
    } else {
      if (req.overwrite) mta_zero_bytes(out_f32, (long)M * ldc * (long)sizeof(float), st);
      dispatch_mode(2, g, ksplit, st);
      if (req.norm_parts) sumsq_parts_kernel<<<NORM_PARTS, 256, 0, st>>>(out_f32, (long)M * ldc, req.norm_parts);
    }
    return 0;
  }
  if (defer == 2) {
    // a weight gradient queued for the grouped launch at mta_gemm_group_flush (too big for the 64 x 64 tiles: now)
    if (!(mode == 2 || (mode == 0 && (flags & EPI_ACCUM)))) return 8;
    // small outputs (the transformer's <= 512 x 512 weights) stay grouped whatever K: at B = 8 (K = 50,176 tokens)
    // the 256 x 256 kernel re-split them ~128 ways into fp32 slabs, and the 16 slab reduces per step cost more than
    // the products (splitk_reduce 35 us each, profiles/r5_transformer_b8_grouped_wgrad.txt)
    if ((big_eligible(g, ksplit) || (long)M * N * K >= (1L << 31)) && (long)M * N > GROUP_SMALL_OUT) {
      dispatch_mode(mode, g, ksplit, st);
      return 0;
    }
    if ((gq.n[0] || gq.n[1]) && gq.st != st) mta_gemm_group_flush();
    const int kind = mode == 2 ? 1 : 0;
    if (gq.n[kind] == GROUP_QMAX) mta_gemm_group_flush();
    gq.g[kind][gq.n[kind]] = g;
    gq.ks[kind][gq.n[kind]] = ksplit;
    ++gq.n[kind];
    gq.st = st;
    return 0;
  }
  if (defer) {
    // a weight-gradient GEMM held back for the next call (its input-gradient partner): one paired launch
    if (!(mode == 2 || (mode == 0 && (flags & EPI_ACCUM)))) return 8;
    mta_gemm_flush();
    pending.on = true;
    pending.mode = mode;
    pending.g = g;
    pending.ksplit = ksplit;
    pending.st = st;
    return 0;
  }
  if (pending.on) {
    pending.on = false;
    const bool same = pending.st == st;
    const bool paired =
        same && ((pending.mode == 2 && mode == 1 && launch_pair(pending.g, pending.ksplit, g, ksplit, st)) ||
                 (pending.mode == 2 && mode == 2 && launch_pair_ww(pending.g, pending.ksplit, g, ksplit, st)) ||
                 (pending.mode == 0 && mode == 0 && (flags & EPI_ACCUM) &&
                  launch_pair_nn_acc(pending.g, pending.ksplit, g, ksplit, st)));
    if (!paired) {
      dispatch_mode(pending.mode, pending.g, pending.ksplit, pending.st);
      dispatch_mode(mode, g, ksplit, st);
    }
    return 0;
  }
  dispatch_mode(mode, g, ksplit, st);
  return 0;
}

}  // namespace

extern "C" int mta_gemm_bf16(int mode, const void* A, const void* B, int M, int N, int K, int lda, int ldb,
                             float alpha, int flags, const float* bias, const float* resid, const void* aux_in,
                             const uint64_t* seed, float drop_p, void* out_bf16, float* out_f32, void* aux_pre,
                             int ldc, int n_store, int ksplit, float* bias_grad, int defer, hipStream_t st) {
  return gemm_bf16_impl(mode, A, B, M, N, K, lda, ldb, alpha, flags, bias, resid, aux_in, seed, drop_p, out_bf16,
                        out_f32, aux_pre, ldc, n_store, ksplit, bias_grad, defer, st);
}

extern "C" void mta_gemm_grad_producer(float* norm_parts, int overwrite) {
  g_producer.norm_parts = norm_parts;
  g_producer.overwrite = overwrite != 0;
}
extern "C" int mta_gemm_norm_parts() { return NORM_PARTS; }
