// MFMA split-K weight gradient of one LSTM layer, shared by the standalone kernel (lstm_aux.hip) and the
// backward stack kernel's fused weight-gradient workgroups (lstm_stack.hip).
#pragma once

#include <cstdlib>

#include "common.h"

#ifndef WG_SLICE_STAMP
#define WG_SLICE_STAMP(k) \
  do {                    \
  } while (0)
#endif

namespace mta_wgrad {

// ---------------------------------------------------------------------------------------------
// weight gradient (MFMA split-K):
//   out[r(c')][c] += sum_rows dG[row][c'] * Bop[row][c],   Bop = [h_{t-1} | layer input]
//   db[r(c')]     += sum_rows dG[row][c']
// Grid: (row chunk) x (quarter of the 4H gate columns c').  A workgroup stages 32-row slices of
// dG (its 64 c') and of both operands through LDS as k-contiguous images (bf16 hi/lo, or fp32 for
// 'highest'), so every MFMA fragment is one ds_read_b128 (bf16) / ds_read_b32 (f32); the next slice's
// global loads are issued into registers before the current slice's MFMAs (register-staged pipeline).
// Each wave owns 16 c' x all (H + Fp) operand columns.  The chunk partials are added with no-return
// f32 atomics straight from the accumulator layout: for a fixed accumulator register the 64 lanes
// cover 4 consecutive gate-major rows x 16 consecutive columns (4 x 64 B segments).
// The per-chunk partial volume (nchunks x 4H x (H+F) floats) is what the chunk count trades
// against per-CU load time; the launcher picks ~30 chunks for T=60.
// ---------------------------------------------------------------------------------------------
constexpr int WG_KS = 32;  // rows per stage (= bf16 MFMA K)
constexpr int WG_MAX_UNITS_PER_THREAD = 2;

template <int PREC>
struct WgImg {
  // row stride of the k-contiguous images, in elements: bf16 32 + 8 pad (80 B), f32 32 + 4 pad (144 B)
  static constexpr int RS = PREC == PREC_F32 ? 36 : 40;
  static constexpr int ESZ = PREC == PREC_F32 ? 4 : 2;
  static constexpr int PLANES = PREC == PREC_BF16X3 ? 2 : 1;
};

struct WgArgs {
  const float* dG;    // (T*Np, 4H) unit-major columns
  const float* hseq;  // (T, Np, H)
  const float* inp;   // layer input: time-major (T*Np, F) or batch-first (N, T, F)
  int inp_batch_first, N, Np, T, H, F, FP, rows_per_chunk, nchunks, lo_off;  // lo_off: lo plane offset (elements)
  float* g_wih;       // (4H, F) gate-major rows
  float* g_whh;       // (4H, H)
  float* g_bih;       // (4H)
  float* g_bhh;       // (4H)
  // deterministic mode: per-chunk partials [chunk][4H (H + F) + 4H] written with plain stores instead of the
  // f32 atomics; wgrad_reduce_kernel adds them to the gradients in chunk order (bit-reproducible runs)
  float* part;
};

__host__ __device__ inline long wg_part_elems(int H, int F) { return 4L * H * (H + F) + 4L * H; }

// time steps per row chunk: the standalone kernel aims at ~30 chunks, the stack kernel's fused workgroups at
// ~60 (short chunks keep the tail after the last layer small)
inline int wg_time_chunk(int T, bool fused) { return fused ? (T + 59) / 60 : (T + 29) / 30; }
inline int wg_nchunks(int T, bool fused) {
  const int tc = wg_time_chunk(T, fused);
  return (T + tc - 1) / tc;
}

// One staging unit = 8 rows x 4 columns of one operand (A = dG, or B = [h_{t-1} | inp]).
struct WgUnit {
  float4 v[8];
  uint32_t mask;  // bit 4*j + c: element (row j, column c) is valid
};

// 16 bytes of data another workgroup of the SAME launch stored write-through (sc1): two 8-byte agent-scope
// atomic loads (global_load_dwordx2 ... sc1), which miss a possibly stale line in this XCD's L2
__device__ __forceinline__ float4 wg_load_sc1(const float* p) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(const_cast<float*>(p));
  const unsigned long long x = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long y = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float4(__builtin_bit_cast(float, (unsigned)x), __builtin_bit_cast(float, (unsigned)(x >> 32)),
                     __builtin_bit_cast(float, (unsigned)y), __builtin_bit_cast(float, (unsigned)(y >> 32)));
}

template <int PREC>
__device__ __forceinline__ void wg_store_unit(char* img, int col0, int k0, const WgUnit& u, int lo_off) {
  using I = WgImg<PREC>;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = c == 0 ? u.v[j].x : c == 1 ? u.v[j].y : c == 2 ? u.v[j].z : u.v[j].w;
    if constexpr (PREC == PREC_F32) {
      float* dst = reinterpret_cast<float*>(img) + (size_t)(col0 + c) * I::RS + k0;
      *reinterpret_cast<float4*>(dst) = make_float4(x[0], x[1], x[2], x[3]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(x[4], x[5], x[6], x[7]);
    } else {
      bf16x8 hi, lo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 h, l;
        split_bf16(x[j], h, l);
        hi[j] = h;
        lo[j] = l;
      }
      __bf16* dst = reinterpret_cast<__bf16*>(img) + (size_t)(col0 + c) * I::RS + k0;
      *reinterpret_cast<bf16x8*>(dst) = hi;
      if constexpr (PREC == PREC_BF16X3) {
        *reinterpret_cast<bf16x8*>(dst + lo_off) = lo;
      }
    }
  }
}

// One workgroup of NWAVES waves: chunk `chunk` of the rows x c' block `quarter` of CQ = 16 NWAVES gate
// columns.  SC1A: the dG rows were produced by other workgroups of the same launch (lstm_stack.hip's fused
// backward) and are read with sc1 loads.
struct WgNoWait {
  __device__ void operator()() const {}
};

// wait(): called once by every thread before the first dG (A operand) load -- the fused backward's chunk-ready poll.
// Chunks of at most four K slices whose units fit one per thread (B = 1..2 windows: a chunk is one step of
// Np <= 128 rows) take the short path: the B operand ([h_{t-1} | inp], which the backward does not write) is loaded
// BEFORE the wait, and the A slices all at once after it -- one load round trip after the chunk is ready instead of
// one per slice (r6 timelines: ~3.5 us per slice, 18.5 us for the chunk of step 0, the whole tail of the backward).
template <int PREC, int NWAVES, bool SC1A, typename Wait = WgNoWait>
__device__ __forceinline__ void wgrad_body(const WgArgs& a, const int chunk, const int quarter, char* lds,
                                           const Wait& wait = Wait()) {
  using I = WgImg<PREC>;
  constexpr int THREADS = 64 * NWAVES;
  constexpr int CQ = 16 * NWAVES;
  // LDS plane: A image (CQ c' rows) then B image (H + FP rows), row stride RS; for bf16x3 the lo plane
  // follows at +lo_off elements.
  const int H = a.H, FP = a.FP, G4 = 4 * H;
  const int NB = H + FP;              // operand columns (multiple of 16)
  const int R = a.T * a.Np;
  const int row_begin = chunk * a.rows_per_chunk;
  const int row_end = min(row_begin + a.rows_per_chunk, R);
  const int cq0 = quarter * CQ;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // staging units: A: 4 row-groups x 16 col-groups; B: 4 x (NB/4)
  const int nA = 4 * (CQ / 4);
  const int nUnits = nA + 4 * (NB / 4);
  char* imgA = lds;
  char* imgB = lds + (size_t)CQ * I::RS * I::ESZ;  // B rows start after the 64 A rows (per plane)

  float bias_acc[4] = {0.f, 0.f, 0.f, 0.f};  // column sums of this thread's A unit (if any)

  // Unit descriptors (fixed for the whole chunk): base pointer, row stride, row shift, valid row range.
  // Loads keep the raw values plus a validity bitmask (bit 4*j + c); the mask is applied only when the
  // unit is written to LDS, one MFMA slice later -- using the data right after the load (a select or a
  // mask multiply) would make every load wait for its own data, serialising the prefetch.
  struct Desc {
    const float* base;
    int stride, shift, row_lo, scalar, col, sc1;  // scalar: element-wise inp path (batch-first or F % 4)
    bool colok;
  };
  auto make_desc = [&](int u) {
    Desc d;
    d.scalar = 0;
    d.sc1 = 0;
    d.shift = 0;
    d.row_lo = row_begin;
    d.colok = true;
    if (u < nA) {
      d.col = (u >> 2) * 4;
      d.base = a.dG + cq0 + d.col;
      d.stride = G4;
      d.sc1 = SC1A ? 1 : 0;
    } else {
      const int col = ((u - nA) >> 2) * 4;
      d.col = col;
      if (col < H) {
        d.base = a.hseq + col;
        d.stride = H;
        d.shift = a.Np;  // h_{t-1}: rows t >= 1 only
        d.row_lo = max(row_begin, a.Np);
      } else {
        const int f0 = col - H;
        d.colok = f0 < a.F;
        d.scalar = (a.inp_batch_first || (a.F & 3)) ? 1 : 0;
        d.base = a.inp + (d.colok && !d.scalar ? f0 : 0);
        d.stride = a.F;
        d.col = f0;
      }
    }
    return d;
  };
  const int u0 = tid, u1 = tid + THREADS;

  auto load_unit = [&](const Desc& d, int u, int k0, WgUnit& out) __attribute__((always_inline)) {
    const int r0 = k0 + (u & 3) * 8;
    uint32_t mask = 0;
    if (SC1A && d.sc1) {  // wave-uniform: the A units fill whole waves (CQ = 16 NWAVES units)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int row = r0 + j;
        const bool ok = (row >= d.row_lo) & (row < row_end);
        out.v[j] = wg_load_sc1(d.base + (size_t)(ok ? row : 0) * d.stride);
        mask |= ok ? 0xFu << (4 * j) : 0u;
      }
    } else if (!d.scalar) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int row = r0 + j;
        const bool ok = (row >= d.row_lo) & (row < row_end) & d.colok;
        const int rr = ok ? row - d.shift : 0;
        out.v[j] = *reinterpret_cast<const float4*>(d.base + (size_t)rr * d.stride);
        mask |= ok ? 0xFu << (4 * j) : 0u;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int row = r0 + j;
        const int t = row / a.Np, n = row - t * a.Np;
        const bool okr = (row < row_end) & (!a.inp_batch_first | (n < a.N));
        float e[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int f = d.col + c;
          const bool ok = okr & (f < a.F);
          const size_t off = a.inp_batch_first ? ((size_t)n * a.T + t) * a.F + f : (size_t)row * a.F + f;
          e[c] = a.inp[ok ? off : 0];
          mask |= ok ? 1u << (4 * j + c) : 0u;
        }
        out.v[j] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
    out.mask = mask;
  };
  auto store_unit = [&](int u, WgUnit& v) __attribute__((always_inline)) {
    const int rg = u & 3;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t m = v.mask >> (4 * j);
      v.v[j].x = (m & 1u) ? v.v[j].x : 0.f;
      v.v[j].y = (m & 2u) ? v.v[j].y : 0.f;
      v.v[j].z = (m & 4u) ? v.v[j].z : 0.f;
      v.v[j].w = (m & 8u) ? v.v[j].w : 0.f;
    }
    if (u < nA) {
      const int cg = u >> 2;
      wg_store_unit<PREC>(imgA, cg * 4, rg * 8, v, a.lo_off);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bias_acc[0] += v.v[j].x;
        bias_acc[1] += v.v[j].y;
        bias_acc[2] += v.v[j].z;
        bias_acc[3] += v.v[j].w;
      }
    } else {
      const int cg = (u - nA) >> 2;
      wg_store_unit<PREC>(imgB, cg * 4, rg * 8, v, a.lo_off);
    }
  };

  // accumulators: this wave's 16 c' x NB columns -> NB/16 tiles (<= 16)
  constexpr int MAX_NT = 16;
  const int NT = NB / 16;
  // a chunk inside step 0 has h_{t-1} = 0: its W_hh tiles (the first H / 16) are all zero -- skip their products
  // and atomics (the step-0 chunk is the one that trails the recurrence)
  const int JT0 = row_end <= a.Np ? H / 16 : 0;
  f32x4 acc[MAX_NT];
#pragma unroll
  for (int j = 0; j < MAX_NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int am = wave * 16 + (lane & 15);
  auto mfma_slice = [&]() __attribute__((always_inline)) {
    if constexpr (PREC == PREC_F32) {
      const float* A = reinterpret_cast<const float*>(imgA);
      const float* B = reinterpret_cast<const float*>(imgB);
#pragma unroll
      for (int k4 = 0; k4 < WG_KS / 4; ++k4) {
        const float av = A[(size_t)am * I::RS + 4 * k4 + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < MAX_NT; ++j) {
          if (j >= JT0 && j < NT) {
            const float bv = B[(size_t)(16 * j + (lane & 15)) * I::RS + 4 * k4 + (lane >> 4)];
            acc[j] = mfma16x16x4f32(av, bv, acc[j]);
          }
        }
      }
    } else {
      const __bf16* A = reinterpret_cast<const __bf16*>(imgA);
      const __bf16* B = reinterpret_cast<const __bf16*>(imgB);
      const size_t lo_off = a.lo_off;
      const bf16x8 ahi = *reinterpret_cast<const bf16x8*>(A + (size_t)am * I::RS + 8 * (lane >> 4));
      bf16x8 alo;
      if constexpr (PREC == PREC_BF16X3) alo = *reinterpret_cast<const bf16x8*>(A + lo_off + (size_t)am * I::RS + 8 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < MAX_NT; ++j) {
        if (j >= JT0 && j < NT) {
          const size_t bo = (size_t)(16 * j + (lane & 15)) * I::RS + 8 * (lane >> 4);
          const bf16x8 bhi = *reinterpret_cast<const bf16x8*>(B + bo);
          acc[j] = mfma16x16x32(ahi, bhi, acc[j]);
          if constexpr (PREC == PREC_BF16X3) {
            const bf16x8 blo = *reinterpret_cast<const bf16x8*>(B + lo_off + bo);
            acc[j] = mfma16x16x32(ahi, blo, acc[j]);
            acc[j] = mfma16x16x32(alo, bhi, acc[j]);
          }
        }
      }
    }
  };

  const int nsl = (row_end - row_begin + WG_KS - 1) / WG_KS;
  const int nB = nUnits - nA;
  // short path: thread t holds A unit t % nA of slice t / nA and B unit t % nB of slice t / nB (its own code: with
  // the pipelined path's descriptors and units live beside its own, the kernel spilled)
  // (deterministic partials keep the pipelined path: there a slice's bias sum would overwrite another's partial)
  const bool shortp = !a.part && nsl <= 4 && nA * nsl <= THREADS && nB * nsl <= THREADS;
  int ubias;      // this thread's A unit (bias column group) and whether it has one
  bool hasbias;
  if (shortp) {
    const int sa = tid / nA, sb = tid / nB;
    const int ua = tid % nA, ub = nA + tid % nB;
    const bool has0 = sa < nsl, has1 = sb < nsl;
    WgUnit st0, st1;
    {
      const Desc db = make_desc(ub);
      if (has1) load_unit(db, ub, row_begin + sb * WG_KS, st1);
    }
    wait();
    {
      const Desc da = make_desc(ua);
      if (has0) load_unit(da, ua, row_begin + sa * WG_KS, st0);
    }
    for (int sl = 0; sl < nsl; ++sl) {
      WG_SLICE_STAMP(sl);
      __syncthreads();  // previous slice's fragment reads are done
      if (has0 && sa == sl) store_unit(ua, st0);
      if (has1 && sb == sl) store_unit(ub, st1);
      __syncthreads();
      mfma_slice();
    }
    ubias = ua;
    hasbias = has0;
  } else {
    const Desc d0 = make_desc(u0 < nUnits ? u0 : 0), d1 = make_desc(u1 < nUnits ? u1 : 0);
    const bool has0 = u0 < nUnits, has1 = u1 < nUnits;
    WgUnit st0, st1;
    wait();
    if (has0) load_unit(d0, u0, row_begin, st0);
    if (has1) load_unit(d1, u1, row_begin, st1);
    int k0 = row_begin;
    for (int sl = 0; k0 < row_end; k0 += WG_KS, ++sl) {
      WG_SLICE_STAMP(sl < 16 ? sl : 15);
      __syncthreads();  // previous slice's fragment reads are done
      if (has0) store_unit(u0, st0);
      if (has1) store_unit(u1, st1);
      __syncthreads();
      const int kn = k0 + WG_KS;
      if (kn < row_end) {  // next slice in flight during this slice's MFMAs
        if (has0) load_unit(d0, u0, kn, st0);
        if (has1) load_unit(d1, u1, kn, st1);
      }
      mfma_slice();
    }
    ubias = u0;
    hasbias = u0 < nA;
  }

  WG_SLICE_STAMP(16);
  // ---- partials -> gradients (no-return f32 atomics) ----
  // D layout: lane holds D[4(l>>4)+i][l&15]; local c' = 16*wave + 4(l>>4) + i  ->  gate g = i, unit u
  const int qrow = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cp = cq0 + wave * 16 + 4 * qrow + i;
    const int r = (cp & 3) * H + (cp >> 2);
#pragma unroll
    for (int j = 0; j < MAX_NT; ++j) {
      if (j < NT && (a.part || j >= JT0)) {  // (deterministic partials: the skipped tiles write their zeros)
        const int col = 16 * j + (lane & 15);
        const float v = acc[j][i];
        if (a.part) {
          if (col < H + a.F) a.part[chunk * wg_part_elems(H, a.F) + (size_t)r * (H + a.F) + col] = v;
        } else if (col < H) {
          atomicAdd(a.g_whh + (size_t)r * H + col, v);
        } else if (col - H < a.F) {
          atomicAdd(a.g_wih + (size_t)r * a.F + (col - H), v);
        }
      }
    }
  }
  WG_SLICE_STAMP(17);
  // bias: reduce the 4 row-group threads of each A column group (lanes t, t^1, t^2, t^3; short path: one sum per
  // slice -- nA is a multiple of 4, so a slice's units stay 4-aligned in the thread index)
  if (hasbias) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float v = bias_acc[c];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      bias_acc[c] = v;
    }
    if ((ubias & 3) == 0) {
      const int cg = ubias >> 2;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cp = cq0 + cg * 4 + c;
        const int r = (cp & 3) * H + (cp >> 2);
        if (a.part) {
          a.part[chunk * wg_part_elems(H, a.F) + 4L * H * (H + a.F) + r] = bias_acc[c];
        } else {
          atomicAdd(a.g_bih + r, bias_acc[c]);
          atomicAdd(a.g_bhh + r, bias_acc[c]);
        }
      }
    }
  }
}


// deterministic mode: gradients += the per-chunk partials summed in chunk order (one thread per element)
static __global__ void wgrad_reduce_kernel(WgArgs a) {
  const long E = wg_part_elems(a.H, a.F);
  const int HF = a.H + a.F;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (long)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int c = 0; c < a.nchunks; ++c) acc += a.part[c * E + e];
    if (e < 4L * a.H * HF) {
      const int r = (int)(e / HF), col = (int)(e % HF);
      if (col < a.H) a.g_whh[(size_t)r * a.H + col] += acc;
      else a.g_wih[(size_t)r * a.F + (col - a.H)] += acc;
    } else {
      const int r = (int)(e - 4L * a.H * HF);
      a.g_bih[r] += acc;
      a.g_bhh[r] += acc;
    }
  }
}

}  // namespace mta_wgrad
