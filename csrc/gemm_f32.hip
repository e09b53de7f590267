// fp32-operand MFMA GEMM for the per-layer LSTM path (ops/lstm.py _LSTMStackFn): the time-parallel input
// projection gx = x W_ih^T + b of deeper layers (and of layer 0 when F is not fused into the recurrence) and
// the input gradient dx = dG W_ih (x the layer's input-dropout mask).  Those were torch.addmm / mm calls, i.e.
// hipBLASLt Cijk kernels at the matmul precision torch happened to have; here they honour the op's own
// precision code like the recurrence kernels do (common.h PREC_*):
//   PREC_F32     v_mfma_f32_16x16x4_f32 on the fp32 operands
//   PREC_BF16X3  every operand split hi + lo in registers, hi*hi + hi*lo + lo*hi (3 x v_mfma_f32_16x16x32_bf16)
//   PREC_BF16    one bf16 pass
//
//   C[M][N] = A[M][K] . B^T (+ bias[N]) (* mask[M][N])      B stored [N][K] (BKN = false) or [K][N] (BKN = true)
//
// 64 x 64 tile per 256-thread workgroup (4 waves in 2 x 2, 32 x 32 = 2 x 2 MFMA blocks each), BK = 32 staged
// through LDS as fp32 rows (k-contiguous, the [K][N] form transposed while staging) with the next k-slice
// prefetched into registers during the current slice's MFMAs.  Shapes are arbitrary (edge tiles zero-fill).
// Reference for the products: cuDNN's LSTM input GEMMs behind `src/model.py:88-94`.
#include "common.h"

namespace {

constexpr int BM = 64, BN = 64, BK = 32, TPB = 256;
constexpr int LS = BK + 4;  // LDS row stride (floats)

struct GemmF32Args {
  const float* A;
  const float* B;
  const float* bias;
  const float* mask;
  float* C;
  int M, N, K;
};

template <bool BKN>
struct Stage {
  float a[8];
  float b[8];
};

template <bool BKN>
__device__ __forceinline__ void load_stage(const GemmF32Args& p, int m0, int n0, int k0, Stage<BKN>& s) {
  const int t = threadIdx.x;
  // A: rows m0 + t/8 (+32), k = k0 + 4 (t%8) .. +3
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int m = m0 + t / 8 + 32 * r, k = k0 + 4 * (t % 8);
#pragma unroll
    for (int e = 0; e < 4; ++e) s.a[4 * r + e] = (m < p.M && k + e < p.K) ? p.A[(size_t)m * p.K + k + e] : 0.f;
  }
  if constexpr (!BKN) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int n = n0 + t / 8 + 32 * r, k = k0 + 4 * (t % 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) s.b[4 * r + e] = (n < p.N && k + e < p.K) ? p.B[(size_t)n * p.K + k + e] : 0.f;
    }
  } else {
    // B[k][n]: k = k0 + t/16 (+16), n = n0 + 4 (t%16) .. +3 (contiguous in memory)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int k = k0 + t / 16 + 16 * r, n = n0 + 4 * (t % 16);
#pragma unroll
      for (int e = 0; e < 4; ++e) s.b[4 * r + e] = (k < p.K && n + e < p.N) ? p.B[(size_t)k * p.N + n + e] : 0.f;
    }
  }
}

template <bool BKN>
__device__ __forceinline__ void store_stage(const Stage<BKN>& s, float (*As)[LS], float (*Bs)[LS]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int row = t / 8 + 32 * r, k = 4 * (t % 8);
    *reinterpret_cast<float4*>(&As[row][k]) = make_float4(s.a[4 * r], s.a[4 * r + 1], s.a[4 * r + 2], s.a[4 * r + 3]);
  }
  if constexpr (!BKN) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = t / 8 + 32 * r, k = 4 * (t % 8);
      *reinterpret_cast<float4*>(&Bs[row][k]) =
          make_float4(s.b[4 * r], s.b[4 * r + 1], s.b[4 * r + 2], s.b[4 * r + 3]);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int k = t / 16 + 16 * r, n = 4 * (t % 16);
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[n + e][k] = s.b[4 * r + e];
    }
  }
}

template <int PREC, bool BKN>
__global__ __launch_bounds__(TPB) void gemm_f32_kernel(GemmF32Args p) {
  __shared__ __attribute__((aligned(16))) float As[BM][LS];
  __shared__ __attribute__((aligned(16))) float Bs[BN][LS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int q = lane >> 4, j = lane & 15;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

  f32x4 acc[2][2];
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stage<BKN> st;
  load_stage<BKN>(p, m0, n0, 0, st);
  for (int k0 = 0; k0 < p.K; k0 += BK) {
    __syncthreads();  // previous slice's fragment reads are done
    store_stage<BKN>(st, As, Bs);
    __syncthreads();
    if (k0 + BK < p.K) load_stage<BKN>(p, m0, n0, k0 + BK, st);  // next slice in flight during the MFMAs
    if constexpr (PREC == PREC_F32) {
#pragma unroll
      for (int s = 0; s < BK / 4; ++s) {
        float av[2], bv[2];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) av[bi] = As[wm * 32 + bi * 16 + j][4 * s + q];
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) bv[bj] = Bs[wn * 32 + bj * 16 + j][4 * s + q];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = mfma16x16x4f32(av[bi], bv[bj], acc[bi][bj]);
      }
    } else {
      bf16x8 ahi[2], alo[2], bhi[2], blo[2];
#pragma unroll
      for (int bi = 0; bi < 2; ++bi) {
        const float4 v0 = *reinterpret_cast<const float4*>(&As[wm * 32 + bi * 16 + j][8 * q]);
        const float4 v1 = *reinterpret_cast<const float4*>(&As[wm * 32 + bi * 16 + j][8 * q + 4]);
        const float xv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          __bf16 hi, lo;
          split_bf16(xv[e], hi, lo);
          ahi[bi][e] = hi;
          alo[bi][e] = lo;
        }
      }
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) {
        const float4 v0 = *reinterpret_cast<const float4*>(&Bs[wn * 32 + bj * 16 + j][8 * q]);
        const float4 v1 = *reinterpret_cast<const float4*>(&Bs[wn * 32 + bj * 16 + j][8 * q + 4]);
        const float xv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          __bf16 hi, lo;
          split_bf16(xv[e], hi, lo);
          bhi[bj][e] = hi;
          blo[bj][e] = lo;
        }
      }
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) {
          if constexpr (PREC == PREC_BF16X3) {
            acc[bi][bj] = mfma16x16x32(alo[bi], bhi[bj], acc[bi][bj]);
            acc[bi][bj] = mfma16x16x32(ahi[bi], blo[bj], acc[bi][bj]);
          }
          acc[bi][bj] = mfma16x16x32(ahi[bi], bhi[bj], acc[bi][bj]);
        }
    }
  }
  // epilogue: + bias, * mask, guarded fp32 stores (lane (q, j): rows 4q..4q+3 of column j of each block)
#pragma unroll
  for (int bj = 0; bj < 2; ++bj) {
    const int n = n0 + wn * 32 + bj * 16 + j;
    if (n >= p.N) continue;
    const float b = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 32 + bi * 16 + 4 * q + i;
        if (m >= p.M) continue;
        float v = acc[bi][bj][i] + b;
        if (p.mask) v *= p.mask[(size_t)m * p.N + n];
        p.C[(size_t)m * p.N + n] = v;
      }
  }
}

template <int PREC>
void launch(const GemmF32Args& p, bool bkn, hipStream_t st) {
  const dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN);
  if (bkn) gemm_f32_kernel<PREC, true><<<grid, TPB, 0, st>>>(p);
  else gemm_f32_kernel<PREC, false><<<grid, TPB, 0, st>>>(p);
}

}  // namespace

extern "C" int mta_gemm_f32(int prec, const float* A, const float* B, const float* bias, const float* mask, float* C,
                            int M, int N, int K, int b_kn, hipStream_t st) {
  if (M < 1 || N < 1 || K < 1 || (size_t)M * N >= (1ull << 40)) return -1;
  GemmF32Args p{A, B, bias, mask, C, M, N, K};
  if (prec == PREC_F16X2) prec = PREC_BF16X3;  // an LSTM-forward mode (bounded activations); general operands: bf16x3
  if (prec == PREC_F32) launch<PREC_F32>(p, b_kn != 0, st);
  else if (prec == PREC_BF16X3) launch<PREC_BF16X3>(p, b_kn != 0, st);
  else if (prec == PREC_BF16) launch<PREC_BF16>(p, b_kn != 0, st);
  else return -1;
  return 0;
}
