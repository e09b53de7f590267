// Time-parallel companions of the LSTM recurrences (csrc/lstm.hip):
//
//   mta_lstm_wgrad   dW_ih, dW_hh, db of one layer from the unit-major dG, accumulated straight into the
//                    parameters' gradient views (the flat gradient buffer): replaces per layer two library
//                    GEMMs (whose single-kernel K=T*Np~7k reductions leave the GPU idle), a bias reduction,
//                    an un-permute gather and four AccumulateGrad adds.
//   mta_lstm_prep    per-step unit-major copies of W_ih and (b_ih + b_hh) for the input-projection GEMM.
//   mta_gather_batch HBM-resident dataset -> static batch buffers, indices from a device permutation and a
//                    device cursor, so batch assembly lives inside the captured train-step graph.
#include "common.h"

namespace {

// ---------------------------------------------------------------------------------------------
// weight gradient:  out[r][c] += sum_rows dG[row][c'(r)] * B[row][c]  (fp32 FMA, exact)
// blockIdx.z selects the operand: 0 = h_{t-1} (dW_hh), 1 = layer input (dW_ih), 2 = ones (db)
// ---------------------------------------------------------------------------------------------
constexpr int WG_THREADS = 256;
constexpr int TM = 64;   // c' (gate-column) tile
constexpr int TN = 64;   // operand-column tile
constexpr int KC = 32;   // rows per LDS stage

__global__ __launch_bounds__(WG_THREADS) void lstm_wgrad_kernel(
    const float* __restrict__ dG,    // (T*Np, 4H) unit-major columns
    const float* __restrict__ hseq,  // (T, Np, H)
    const float* __restrict__ inp,   // layer input: time-major (T*Np, F) or batch-first (N, T, F)
    int inp_batch_first, int N, int Np, int T, int H, int F, int rows_per_block,
    float* __restrict__ g_wih,       // (4H, F) gate-major rows
    float* __restrict__ g_whh,       // (4H, H)
    float* __restrict__ g_bih,       // (4H)
    float* __restrict__ g_bhh) {     // (4H)
  __shared__ __attribute__((aligned(16))) float As[KC][TM + 4];
  __shared__ __attribute__((aligned(16))) float Bs[KC][TN + 4];
  const int G4 = 4 * H;
  const int which = blockIdx.z;
  const int C = which == 0 ? H : (which == 1 ? F : 1);
  const int m0 = blockIdx.y * TM;           // c' tile
  const int n0 = blockIdx.x % ((C + TN - 1) / TN) * TN;
  const int kblk = blockIdx.x / ((C + TN - 1) / TN);
  if (n0 >= C) return;
  const int R = T * Np;
  const int row_begin = (which == 0 ? Np : 0) + kblk * rows_per_block;  // dW_hh: rows t >= 1 only
  const int row_end = min(row_begin + rows_per_block, R);
  if (row_begin >= row_end) return;

  const int tid = threadIdx.x;
  const int tm = (tid & 15) * 4;   // 4 c' per thread
  const int tn = (tid >> 4) * 4;   // 4 columns per thread
  float acc[4][4] = {};

  for (int k0 = row_begin; k0 < row_end; k0 += KC) {
    // stage dG rows [k0, k0+KC) x c' [m0, m0+TM) and operand rows x cols [n0, n0+TN)
    for (int e = tid; e < KC * TM; e += WG_THREADS) {
      const int kr = e / TM, mc = e % TM;
      const int row = k0 + kr;
      As[kr][mc] = (row < row_end && m0 + mc < G4) ? dG[(size_t)row * G4 + m0 + mc] : 0.f;
    }
    for (int e = tid; e < KC * TN; e += WG_THREADS) {
      const int kr = e / TN, nc = e % TN;
      const int row = k0 + kr;
      float v = 0.f;
      if (row < row_end && n0 + nc < C) {
        if (which == 0) {
          v = hseq[(size_t)(row - Np) * H + n0 + nc];  // h_{t-1} for row (t, n)
        } else if (which == 1) {
          if (inp_batch_first) {
            const int t = row / Np, n = row % Np;
            v = n < N ? inp[((size_t)n * T + t) * F + n0 + nc] : 0.f;
          } else {
            v = inp[(size_t)row * F + n0 + nc];
          }
        } else {
          v = 1.f;
        }
      }
      Bs[kr][nc] = v;
    }
    __syncthreads();
#pragma unroll 4
    for (int kr = 0; kr < KC; ++kr) {
      const float4 a = *reinterpret_cast<const float4*>(&As[kr][tm]);
      const float4 b = *reinterpret_cast<const float4*>(&Bs[kr][tn]);
      const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[i][jj] = fmaf(av[i], bv[jj], acc[i][jj]);
    }
    __syncthreads();
  }
  // scatter-add into gate-major rows: c' = 4u + g  ->  r = g*H + u
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cp = m0 + tm + i;
    if (cp >= G4) continue;
    const int r = (cp & 3) * H + (cp >> 2);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int c = n0 + tn + jj;
      if (c >= C) continue;
      if (which == 0) atomicAdd(&g_whh[(size_t)r * H + c], acc[i][jj]);
      else if (which == 1) atomicAdd(&g_wih[(size_t)r * F + c], acc[i][jj]);
      else if (jj == 0) {
        atomicAdd(&g_bih[r], acc[i][0]);
        atomicAdd(&g_bhh[r], acc[i][0]);
      }
    }
  }
}

// unit-major W_ih (4H, F) and combined bias: row c' = 4u + g  <-  r = g*H + u
__global__ void lstm_prep_kernel(const float* __restrict__ w_ih, const float* __restrict__ b_ih,
                                 const float* __restrict__ b_hh, int H, int F, float* __restrict__ w_um,
                                 float* __restrict__ b_um) {
  const int G4 = 4 * H;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < G4 * F; e += gridDim.x * blockDim.x) {
    const int cp = e / F, f = e % F;
    const int r = (cp & 3) * H + (cp >> 2);
    w_um[e] = w_ih[(size_t)r * F + f];
  }
  for (int cp = blockIdx.x * blockDim.x + threadIdx.x; cp < G4; cp += gridDim.x * blockDim.x) {
    const int r = (cp & 3) * H + (cp >> 2);
    b_um[cp] = b_ih[r] + b_hh[r];
  }
}

// ---------------------------------------------------------------------------------------------
// batch gather: block (b, k) copies row perm[cursor*B + b] of tensor k into dst_k[b]; the last block
// to finish advances the cursor (every block reads it before arriving, so the update is race-free)
// ---------------------------------------------------------------------------------------------
struct GatherArgs {
  const float* src[4];
  float* dst[4];
  long row_floats[4];
  int ntensors;
};

__global__ void gather_batch_kernel(GatherArgs a, const int* __restrict__ perm, int* cursor, int* arrive, int B,
                                    int row_offset) {
  const int b = blockIdx.x, k = blockIdx.y;
  const int idx = perm[cursor[0] * B + b] + row_offset;
  const long n = a.row_floats[k];
  const float* s = a.src[k] + (size_t)idx * n;
  float* d = a.dst[k] + (size_t)b * n;
  if ((n & 3) == 0 && ((((uintptr_t)s) | ((uintptr_t)d)) & 15) == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(s);
    float4* d4 = reinterpret_cast<float4*>(d);
    for (long i = threadIdx.x; i < n / 4; i += blockDim.x) d4[i] = s4[i];
  } else {
    for (long i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int total = gridDim.x * gridDim.y;
    const int prev = atomicAdd(arrive, 1);
    if (prev == total - 1) {
      arrive[0] = 0;
      cursor[0] = cursor[0] + 1;
    }
  }
}

}  // namespace

extern "C" void mta_lstm_wgrad(const float* dG, const float* hseq, const float* inp, int inp_batch_first, int N,
                               int Np, int T, int H, int F, float* g_wih, float* g_whh, float* g_bih, float* g_bhh,
                               hipStream_t st) {
  const int R = T * Np;
  // ~2 rows-blocks per CU for the widest operand: balance atomics (one slab per block) vs parallelism
  int kblocks = (R + 255) / 256;
  if (kblocks > 64) kblocks = 64;
  int rows_per_block = (R + kblocks - 1) / kblocks;
  rows_per_block = (rows_per_block + KC - 1) / KC * KC;
  kblocks = (R + rows_per_block - 1) / rows_per_block;
  const int cmax = H > F ? H : F;
  dim3 grid(kblocks * ((cmax + TN - 1) / TN), (4 * H + TM - 1) / TM, 3);
  lstm_wgrad_kernel<<<grid, WG_THREADS, 0, st>>>(dG, hseq, inp, inp_batch_first, N, Np, T, H, F, rows_per_block,
                                                 g_wih, g_whh, g_bih, g_bhh);
}

extern "C" void mta_lstm_prep(const float* w_ih, const float* b_ih, const float* b_hh, int H, int F, float* w_um,
                              float* b_um, hipStream_t st) {
  lstm_prep_kernel<<<64, 256, 0, st>>>(w_ih, b_ih, b_hh, H, F, w_um, b_um);
}

extern "C" void mta_gather_batch(const float* const* src, float* const* dst, const long* row_floats, int ntensors,
                                 const int* perm, int* cursor, int* arrive, int B, int row_offset, hipStream_t st) {
  GatherArgs a{};
  for (int k = 0; k < ntensors && k < 4; ++k) {
    a.src[k] = src[k];
    a.dst[k] = dst[k];
    a.row_floats[k] = row_floats[k];
  }
  a.ntensors = ntensors;
  gather_batch_kernel<<<dim3(B, ntensors), 256, 0, st>>>(a, perm, cursor, arrive, B, row_offset);
}
