// Time-parallel companions of the LSTM recurrences (csrc/lstm.hip):
//
//   mta_lstm_wgrad   dW_ih, dW_hh, db of one layer from the unit-major dG, accumulated straight into the
//                    parameters' gradient views (the flat gradient buffer): replaces per layer two library
//                    GEMMs (whose single-kernel K=T*Np~7k reductions leave the GPU idle), a bias reduction,
//                    an un-permute gather and four AccumulateGrad adds.
//   mta_lstm_prep    per-step unit-major copies of W_ih and (b_ih + b_hh) for the input-projection GEMM.
//   mta_gather_batch HBM-resident dataset -> static batch buffers, indices from a device permutation and a
//                    device cursor, so batch assembly lives inside the captured train-step graph.
#include <cstdlib>

#include "common.h"
#include "lstm_wgrad.h"

namespace {

using namespace mta_wgrad;
constexpr int WG_WAVES = 4;
constexpr int WG_THREADS = 64 * WG_WAVES;
constexpr int CQ = 16 * WG_WAVES;

template <int PREC>
__global__ __launch_bounds__(WG_THREADS) void lstm_wgrad_kernel(WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // XCD-aware mapping: the c'-blocks of a chunk run on the same XCD (they share the operand rows)
  const int nq = 4 * a.H / CQ;
  const int b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3;
  const int quarter = slot % nq;
  const int chunk = (slot / nq) * 8 + xcd;
  if (chunk >= a.nchunks) return;
  wgrad_body<PREC, WG_WAVES, false>(a, chunk, quarter, lds);
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
// batch gather: row perm[cursor*B + b] of tensor k -> dst_k[b].  Every (b, k) row is split over
// GATHER_CHUNK-float4 pieces, `span` pieces per block (grid.x = B * chunks of the longest row, grid.y = tensors,
// ~512 blocks), so all of a step's loads are in flight at once (one 256-thread block per 16 KB at B = 1: a 72 KB
// window row took 10 us as one block's serial loop, r2 kernel trace).  Blocks past a shorter row's end only arrive.  The last block
// to arrive advances the cursor (every block reads it before arriving, so the update is race-free).
// ---------------------------------------------------------------------------------------------
constexpr int GATHER_TPB = 256;
constexpr int GATHER_SUBS = 64;        // arrival sub-counters
constexpr int GATHER_SUB_STRIDE = 32;  // ints between counters: the arrive buffer holds (1 + GATHER_SUBS) x 32 words
constexpr int GATHER_CHUNK = GATHER_TPB * 4;  // float4 per block

struct GatherArgs {
  const float* src[4];
  float* dst[4];
  long row_floats[4];
  int ntensors;
  int chunks;  // blocks per row (of the longest row)
  int span;    // GATHER_CHUNK pieces per block
};

__global__ __launch_bounds__(GATHER_TPB) void gather_batch_kernel(GatherArgs a, const int* __restrict__ perm,
                                                                  int* cursor, int* arrive, int B, int row_offset) {
  const int b = blockIdx.x / a.chunks, chunk = blockIdx.x % a.chunks, k = blockIdx.y;
  const int idx = perm[cursor[0] * B + b] + row_offset;
  const long n = a.row_floats[k];
  const float* s = a.src[k] + (size_t)idx * n;
  float* d = a.dst[k] + (size_t)b * n;
  if ((n & 3) == 0 && ((((uintptr_t)s) | ((uintptr_t)d)) & 15) == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(s);
    float4* d4 = reinterpret_cast<float4*>(d);
    for (int piece = chunk * a.span; piece < (chunk + 1) * a.span; ++piece) {
      const long lo = (long)piece * GATHER_CHUNK, hi = lo + GATHER_CHUNK < n / 4 ? lo + GATHER_CHUNK : n / 4;
      if (lo >= hi) break;
      // unconditional loads (clamped index): a guarded load makes hipcc branch around it and wait for each one
      float4 v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long i = lo + r * GATHER_TPB + threadIdx.x;
        v[r] = s4[i < hi ? i : hi - 1];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long i = lo + r * GATHER_TPB + threadIdx.x;
        if (i < hi) d4[i] = v[r];
      }
    }
  } else {
    const long lo = (long)chunk * a.span * GATHER_CHUNK * 4;
    const long hi = lo + (long)a.span * GATHER_CHUNK * 4 < n ? lo + (long)a.span * GATHER_CHUNK * 4 : n;
    for (long i = lo + threadIdx.x; i < hi; i += GATHER_TPB) d[i] = s[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // two-level arrival: block i adds to sub-counter 1 + i % 64, the last of each sub-counter to the top word, the
    // last of those advances the cursor -- ~32 adds per word instead of all ~2,048 on one (same-word atomics
    // serialise at the memory side: the one-word form was ~20 us of the mlp_large B = 64 gather)
    const int total = gridDim.x * gridDim.y;
    const int bid = blockIdx.y * gridDim.x + blockIdx.x;
    const int g = bid % GATHER_SUBS;
    const int gsize = (total - g + GATHER_SUBS - 1) / GATHER_SUBS;
    int* sub = arrive + GATHER_SUB_STRIDE * (1 + g);  // one 128-B line per sub-counter (same-line atomics serialise)
    if (atomicAdd(sub, 1) == gsize - 1) {
      sub[0] = 0;
      const int ng = total < GATHER_SUBS ? total : GATHER_SUBS;
      if (atomicAdd(arrive, 1) == ng - 1) {
        arrive[0] = 0;
        cursor[0] = cursor[0] + 1;
      }
    }
  }
}

}  // namespace

extern "C" int mta_lstm_wgrad(int prec, const float* dG, const float* hseq, const float* inp, int inp_batch_first,
                              int N, int Np, int T, int H, int F, float* g_wih, float* g_whh, float* g_bih,
                              float* g_bhh, float* part, hipStream_t st) {
  if (prec == PREC_F16X2) prec = PREC_BF16X3;
  WgArgs a;
  a.part = part;
  a.dG = dG;
  a.hseq = hseq;
  a.inp = inp;
  a.inp_batch_first = inp_batch_first;
  a.N = N;
  a.Np = Np;
  a.T = T;
  a.H = H;
  a.F = F;
  a.FP = (F + 15) / 16 * 16;
  a.g_wih = g_wih;
  a.g_whh = g_whh;
  a.g_bih = g_bih;
  a.g_bhh = g_bhh;
  const int NB = H + a.FP;
  if (H % 16 || (4 * H) % CQ || NB / 16 > 16 || 4 * (CQ / 4) + NB > WG_MAX_UNITS_PER_THREAD * WG_THREADS) return 1;
  const int tc = wg_time_chunk(T, false);
  a.rows_per_chunk = tc * Np;
  a.nchunks = (T * Np + a.rows_per_chunk - 1) / a.rows_per_chunk;
  const int groups = (a.nchunks + 7) / 8;            // chunk groups of 8 (one per XCD)
  const int blocks = groups * 8 * (4 * H / CQ);      // x c' blocks of 64
  if (prec == PREC_F32) {
    a.lo_off = 0;
    const size_t bytes = (size_t)(CQ + NB) * WgImg<PREC_F32>::RS * 4;
    lstm_wgrad_kernel<PREC_F32><<<blocks, WG_THREADS, bytes, st>>>(a);
  } else {
    a.lo_off = (CQ + NB) * WgImg<PREC_BF16>::RS;
    const size_t plane = (size_t)a.lo_off * 2;
    if (prec == PREC_BF16X3) lstm_wgrad_kernel<PREC_BF16X3><<<blocks, WG_THREADS, 2 * plane, st>>>(a);
    else lstm_wgrad_kernel<PREC_BF16><<<blocks, WG_THREADS, plane, st>>>(a);
  }
  if (part) wgrad_reduce_kernel<<<(int)((wg_part_elems(H, F) + 255) / 256), 256, 0, st>>>(a);
  return 0;
}

// floats of the deterministic-mode partial buffer of one layer (fused: the stack kernel's chunking)
extern "C" long mta_lstm_wgrad_part_floats(int fused, int T, int H, int F) {
  return (long)wg_nchunks(T, fused != 0) * wg_part_elems(H, F);
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
  long longest = 1;
  for (int k = 0; k < ntensors && k < 4; ++k) longest = row_floats[k] > longest ? row_floats[k] : longest;
  const int pieces = (int)((longest + 4L * GATHER_CHUNK - 1) / (4L * GATHER_CHUNK));
  // every block arrives on one counter (the last advances the cursor): keep the grid near 2048 workgroups -- at
  // B = 64 one block per 16-KB piece was ~5k same-word atomics, ~35 us per step; mlp_large B = 64 gather with a
  // target of 512 / 2048 / 8192 blocks: 27.1 / 23.6 / 23.4 us (r3 traces)
  constexpr int grid_target = 2048;
  const int per = B * (ntensors > 0 ? ntensors : 1);
  const int target = grid_target / per > 1 ? grid_target / per : 1;
  a.span = (pieces + target - 1) / target;
  a.chunks = (pieces + a.span - 1) / a.span;
  gather_batch_kernel<<<dim3(B * a.chunks, ntensors), GATHER_TPB, 0, st>>>(a, perm, cursor, arrive, B, row_offset);
}
