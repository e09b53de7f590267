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
// The same kernel is the 32-true GEMM of the MLP / transformer extras (ops/extras.py, `trainer=fast`): A may be
// stored transposed ([K][M], AKM: the weight gradient dY^T X reads dY as stored), rows have their own strides, and
// the epilogue adds the bias, applies GELU (saving its fp32 input), or accumulates into C (the flat fp32 gradient
// buffer) over the first n_store columns.
//
// 64 x 64 tile per 256-thread workgroup (4 waves in 2 x 2, 32 x 32 = 2 x 2 MFMA blocks each), BK = 32 staged
// through LDS as fp32 rows (k-contiguous, the [K][N] form transposed while staging) with the next k-slice
// prefetched into registers during the current slice's MFMAs.  Shapes are arbitrary (edge tiles zero-fill).
// Reference for the products: cuDNN's LSTM input GEMMs behind `src/model.py:88-94`.
#include "common.h"

namespace {

constexpr int BM = 64, BN = 64, BK = 32, TPB = 256;
constexpr int LS = BK + 4;  // LDS row stride (floats)

// epilogue flags (the EPI_* values of gemm.hip): + bias, GELU (input saved to pre), x GELU'(pre) (the input gradient of
// a GELU layer: pre is read), C += instead of C =, + resid[m][n] (row stride ldc: a residual connection)
// a counter-hash dropout scale (0 or 1 / (1 - p)) regenerated from the seed, forward and backward alike
constexpr int F32X_BIAS = 1, F32X_GELU = 2, F32X_DGELU = 4, F32X_ACCUM = 8, F32X_RESID = 16, F32X_DROPOUT = 32;

struct GemmF32Args {
  const float* A;
  const float* B;
  const float* bias;
  const float* mask;
  float* C;
  float* pre;    // F32X_GELU: the GELU input [M][ldc] (or null); F32X_DGELU: read
  const float* resid;  // F32X_RESID: added to the product [M][ldc]
  const uint64_t* seed;  // F32X_DROPOUT: the site's device-resident seed (mta_dropout_scale(seed, m, n, p))
  float drop_p;
  int M, N, K;
  int lda, ldb, ldc, n_store, flags;
};

struct Stage {
  float a[8];
  float b[8];
};

template <bool AKM, bool BKN>
__device__ __forceinline__ void load_stage(const GemmF32Args& p, int m0, int n0, int k0, Stage& s) {
  const int t = threadIdx.x;
  if constexpr (!AKM) {
    // A[m][k]: rows m0 + t/8 (+32), k = k0 + 4 (t%8) .. +3
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int m = m0 + t / 8 + 32 * r, k = k0 + 4 * (t % 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) s.a[4 * r + e] = (m < p.M && k + e < p.K) ? p.A[(size_t)m * p.lda + k + e] : 0.f;
    }
  } else {
    // A stored [k][m]: k = k0 + t/16 (+16), m = m0 + 4 (t%16) .. +3 (contiguous in memory)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int k = k0 + t / 16 + 16 * r, m = m0 + 4 * (t % 16);
#pragma unroll
      for (int e = 0; e < 4; ++e) s.a[4 * r + e] = (k < p.K && m + e < p.M) ? p.A[(size_t)k * p.lda + m + e] : 0.f;
    }
  }
  if constexpr (!BKN) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int n = n0 + t / 8 + 32 * r, k = k0 + 4 * (t % 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) s.b[4 * r + e] = (n < p.N && k + e < p.K) ? p.B[(size_t)n * p.ldb + k + e] : 0.f;
    }
  } else {
    // B[k][n]: k = k0 + t/16 (+16), n = n0 + 4 (t%16) .. +3 (contiguous in memory)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int k = k0 + t / 16 + 16 * r, n = n0 + 4 * (t % 16);
#pragma unroll
      for (int e = 0; e < 4; ++e) s.b[4 * r + e] = (k < p.K && n + e < p.N) ? p.B[(size_t)k * p.ldb + n + e] : 0.f;
    }
  }
}

template <bool AKM, bool BKN>
__device__ __forceinline__ void store_stage(const Stage& s, float (*As)[LS], float (*Bs)[LS]) {
  const int t = threadIdx.x;
  if constexpr (!AKM) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = t / 8 + 32 * r, k = 4 * (t % 8);
      *reinterpret_cast<float4*>(&As[row][k]) =
          make_float4(s.a[4 * r], s.a[4 * r + 1], s.a[4 * r + 2], s.a[4 * r + 3]);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int k = t / 16 + 16 * r, m = 4 * (t % 16);
#pragma unroll
      for (int e = 0; e < 4; ++e) As[m + e][k] = s.a[4 * r + e];
    }
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

template <int PREC, bool AKM, bool BKN>
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

  Stage st;
  load_stage<AKM, BKN>(p, m0, n0, 0, st);
  for (int k0 = 0; k0 < p.K; k0 += BK) {
    __syncthreads();  // previous slice's fragment reads are done
    store_stage<AKM, BKN>(st, As, Bs);
    __syncthreads();
    if (k0 + BK < p.K) load_stage<AKM, BKN>(p, m0, n0, k0 + BK, st);  // next slice in flight during the MFMAs
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
  // epilogue: + bias, GELU (input saved), x GELU'(pre), * mask, * dropout, + resid, = or += guarded fp32 stores (lane (q, j): rows 4q..4q+3 of column
  // j of each block)
#pragma unroll
  for (int bj = 0; bj < 2; ++bj) {
    const int n = n0 + wn * 32 + bj * 16 + j;
    if (n >= p.n_store) continue;
    const float b = (p.flags & F32X_BIAS) && p.bias ? p.bias[n] : 0.f;
    const uint64_t sd = (p.flags & F32X_DROPOUT) ? *p.seed : 0;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 32 + bi * 16 + 4 * q + i;
        if (m >= p.M) continue;
        float v = acc[bi][bj][i] + b;
        const size_t o = (size_t)m * p.ldc + n;
        if (p.flags & F32X_GELU) {
          if (p.pre) p.pre[o] = v;
          v = mta_gelu(v);
        }
        if (p.flags & F32X_DGELU) v *= mta_gelu_grad(p.pre[o]);
        if (p.mask) v *= p.mask[(size_t)m * p.N + n];
        if (p.flags & F32X_DROPOUT) v *= mta_dropout_scale(sd, m, n, p.drop_p);
        if (p.flags & F32X_RESID) v += p.resid[o];
        if (p.flags & F32X_ACCUM) p.C[o] += v;
        else p.C[o] = v;
      }
  }
}

// out[n] += sum over the M rows of A[m][n] (lda): the bias gradients of the 32-true extras.  64 columns per
// workgroup (lane = column: coalesced 256-B rows), its 4 waves take every 4th row with 4 partial sums in flight, the
// wave partials are added in wave order (bit-reproducible)
__global__ __launch_bounds__(256) void colsum_f32_kernel(const float* __restrict__ A, int M, int N, int lda,
                                                         float* __restrict__ out) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + lane;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    int m = wave;
    for (; m + 12 < M; m += 16) {
#pragma unroll
      for (int r = 0; r < 4; ++r) s[r] += A[(size_t)(m + 4 * r) * lda + n];
    }
    for (; m < M; m += 4) s[0] += A[(size_t)m * lda + n];
  }
  part[wave][lane] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  if (wave == 0 && n < N) out[n] += (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
}

template <int PREC>
void launch(const GemmF32Args& p, bool akm, bool bkn, hipStream_t st) {
  const dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN);
  if (akm) {
    if (bkn) gemm_f32_kernel<PREC, true, true><<<grid, TPB, 0, st>>>(p);
    else gemm_f32_kernel<PREC, true, false><<<grid, TPB, 0, st>>>(p);
  } else {
    if (bkn) gemm_f32_kernel<PREC, false, true><<<grid, TPB, 0, st>>>(p);
    else gemm_f32_kernel<PREC, false, false><<<grid, TPB, 0, st>>>(p);
  }
}

int dispatch(int prec, const GemmF32Args& p, bool akm, bool bkn, hipStream_t st) {
  if (prec == PREC_F16X2) prec = PREC_BF16X3;  // an LSTM-forward mode (bounded activations); general operands: bf16x3
  if (prec == PREC_F32) launch<PREC_F32>(p, akm, bkn, st);
  else if (prec == PREC_BF16X3) launch<PREC_BF16X3>(p, akm, bkn, st);
  else if (prec == PREC_BF16) launch<PREC_BF16>(p, akm, bkn, st);
  else return -1;
  return 0;
}

}  // namespace

extern "C" int mta_gemm_f32(int prec, const float* A, const float* B, const float* bias, const float* mask, float* C,
                            int M, int N, int K, int b_kn, hipStream_t st) {
  if (M < 1 || N < 1 || K < 1 || (size_t)M * N >= (1ull << 40)) return -1;
  GemmF32Args p{A, B, bias, mask, C, nullptr, nullptr, nullptr, 0.f, M, N, K, K, b_kn ? N : K, N, N,
                bias ? F32X_BIAS : 0};
  return dispatch(prec, p, false, b_kn != 0, st);
}

// the general form: A [M][K] (lda) or stored [K][M] (a_km); B [N][K] or [K][N] (b_kn) (ldb); C [M][ldc], the first
// n_store columns written; flags F32X_*; pre (F32X_GELU / F32X_DGELU): the GELU input [M][ldc]; mask [M][N]
// (dropout scale: 0 or 1 / (1 - p)) multiplies the result, as does the seed's hash mask (F32X_DROPOUT, rate drop_p);
// resid (F32X_RESID) [M][ldc] is added to it
extern "C" int mta_gemm_f32x(int prec, const float* A, int a_km, int lda, const float* B, int b_kn, int ldb,
                             float* C, int ldc, int n_store, int M, int N, int K, int flags, const float* bias,
                             float* pre, const float* mask, const float* resid, const uint64_t* seed, float drop_p,
                             hipStream_t st) {
  if (M < 1 || N < 1 || K < 1 || (size_t)M * N >= (1ull << 40) || n_store < 1 || n_store > N || ldc < n_store ||
      lda < (a_km ? M : K) || ldb < (b_kn ? N : K) || ((flags & F32X_DGELU) && !pre) || ((flags & F32X_RESID) && !resid) ||
      ((flags & F32X_DROPOUT) && (!seed || !(drop_p >= 0.f && drop_p < 1.f))))
    return -1;
  GemmF32Args p{A, B, bias, mask, C, pre, resid, seed, drop_p, M, N, K, lda, ldb, ldc, n_store, flags};
  return dispatch(prec, p, a_km != 0, b_kn != 0, st);
}

extern "C" void mta_colsum_f32(const float* A, int M, int N, int lda, float* out, hipStream_t st) {
  colsum_f32_kernel<<<(N + 63) / 64, 256, 0, st>>>(A, M, N, lda, out);
}
