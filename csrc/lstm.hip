// Persistent single-layer LSTM recurrences for MI355X (gfx950).
//
// Replaces the reference's cuDNN LSTM (src/model.py:88-94,104).
// Design (one workgroup = 16 sequences = one MFMA M-tile, one wave per 16 hidden units):
//   * time-major activations (T, N, .) so each step's 16-sequence slab is contiguous and the
//     weight-gradient GEMMs need no copies (h_{t-1} is a contiguous prefix);
//   * W_hh lives in VGPRs for the whole sequence as MFMA B fragments (hi/lo bf16 for 'high',
//     f32 for 'highest'); the recurrent state crosses waves through a double-buffered LDS
//     image, so each timestep costs one __syncthreads;
//   * wave w owns units [16w, 16w+16) for all four gates, so the MFMA C/D layout
//     (col = lane&15 -> unit, row = 4*(lane>>4)+reg -> sequence) puts i,f,g,o of one
//     (sequence, unit) in one lane: the cell update is lane-local;
//   * forward stores the activated gates (overwriting the input projection in place) and c_t
//     for BPTT; backward overwrites the gates with dG (pre-activation gradients) which the
//     weight-gradient GEMMs consume.
#include "common.h"

namespace {

constexpr int S = 16;  // sequences per workgroup (MFMA M tile)

// ---------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------
template <int H, int PREC, int FIN>
__global__ __launch_bounds__((H / 16) * 64) void lstm_fwd_kernel(
    const float* __restrict__ x,     // FIN > 0: (N, T, FIN) batch-first layer input
    const float* __restrict__ w_ih,  // FIN > 0: (4H, FIN)
    const float* __restrict__ b_ih,  // FIN > 0: (4H)
    const float* __restrict__ b_hh,  // FIN > 0: (4H)
    const float* gx,                 // FIN == 0: (T, N, 4H) input projection incl. both biases
    float* gates,                    // (T, N, 4H) out: activated [i, f, g, o]; may alias gx
    const float* __restrict__ w_hh,  // (4H, H)
    float* __restrict__ hseq,        // (T, N, H)
    float* __restrict__ cseq,        // (T, N, H)
    int N, int T) {
  constexpr int G4 = 4 * H;
  constexpr int KB = H / 32;  // bf16 k-blocks of 32
  constexpr int KF = H / 4;   // f32 k-steps of 4
  constexpr int ROWB = H + 8; // padded bf16 row (16 B pad)
  constexpr int ROWF = H + 4; // padded f32 row

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int q = lane >> 4, j = lane & 15;
  const int u = 16 * w + j;
  const int n0 = blockIdx.x * S;

  __shared__ __attribute__((aligned(16))) __bf16 h_hi[2][S][ROWB];
  __shared__ __attribute__((aligned(16))) __bf16 h_lo[2][S][ROWB];
  __shared__ __attribute__((aligned(16))) float h_f[2][S][ROWF];

  // ---- weights -> registers -------------------------------------------------------------
  bf16x8 Bhi[4][KB > 0 ? KB : 1], Blo[4][KB > 0 ? KB : 1];
  float Bf[4][PREC == PREC_F32 ? KF : 1];
  if constexpr (PREC == PREC_F32) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int kk = 0; kk < KF; ++kk) Bf[g][kk] = w_hh[(size_t)(g * H + u) * H + 4 * kk + q];
  } else {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float v = w_hh[(size_t)(g * H + u) * H + 32 * kb + 8 * q + e];
          __bf16 hi, lo;
          split_bf16(v, hi, lo);
          Bhi[g][kb][e] = hi;
          Blo[g][kb][e] = lo;
        }
  }
  float wi[4][FIN > 0 ? FIN : 1], bias[4];
  if constexpr (FIN > 0) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bias[g] = b_ih[g * H + u] + b_hh[g * H + u];
#pragma unroll
      for (int f = 0; f < FIN; ++f) wi[g][f] = w_ih[(g * H + u) * FIN + f];
    }
  }

  // ---- zero initial state (buffer 0) ------------------------------------------------------
  for (int idx = threadIdx.x; idx < S * ROWB; idx += blockDim.x) {
    (&h_hi[0][0][0])[idx] = (__bf16)0.f;
    (&h_lo[0][0][0])[idx] = (__bf16)0.f;
  }
  for (int idx = threadIdx.x; idx < S * ROWF; idx += blockDim.x) (&h_f[0][0][0])[idx] = 0.f;
  __syncthreads();

  float c[4] = {0.f, 0.f, 0.f, 0.f};
  bool valid[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) valid[i] = (n0 + 4 * q + i) < N;

  // prefetch input contribution for t = 0
  float nxt[4][4];
  auto load_in = [&](int t, float (&dst)[4][4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + 4 * q + i;
      if constexpr (FIN == 0) {
#pragma unroll
        for (int g = 0; g < 4; ++g) dst[g][i] = valid[i] ? gx[((size_t)t * N + n) * G4 + g * H + u] : 0.f;
      } else {
        float xv[FIN];
#pragma unroll
        for (int f = 0; f < FIN; ++f) xv[f] = valid[i] ? x[((size_t)n * T + t) * FIN + f] : 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float a = bias[g];
#pragma unroll
          for (int f = 0; f < FIN; ++f) a = fmaf(xv[f], wi[g][f], a);
          dst[g][i] = a;
        }
      }
    }
  };
  load_in(0, nxt);

  for (int t = 0; t < T; ++t) {
    const int cur = t & 1;
    f32x4 acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = f32x4{nxt[g][0], nxt[g][1], nxt[g][2], nxt[g][3]};
    if (t + 1 < T) load_in(t + 1, nxt);

    // ---- recurrent MFMA: acc[g] += h_{t-1} (16 x H) . W_hh[g]^T (H x 16) -----------------
    if constexpr (PREC == PREC_F32) {
      const float* hrow = &h_f[cur][j][q * KF];
#pragma unroll
      for (int kk = 0; kk < KF; ++kk) {
        const float a = hrow[kk];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = mfma16x16x4f32(a, Bf[g][kk], acc[g]);
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const bf16x8 ahi = *reinterpret_cast<const bf16x8*>(&h_hi[cur][j][32 * kb + 8 * q]);
        if constexpr (PREC == PREC_BF16X3) {
          const bf16x8 alo = *reinterpret_cast<const bf16x8*>(&h_lo[cur][j][32 * kb + 8 * q]);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            acc[g] = mfma16x16x32(alo, Bhi[g][kb], acc[g]);
            acc[g] = mfma16x16x32(ahi, Blo[g][kb], acc[g]);
          }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = mfma16x16x32(ahi, Bhi[g][kb], acc[g]);
      }
    }

    // ---- gates + cell update (lane-local) ------------------------------------------------
    const int nb = (t + 1) & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float ig = mta_sigmoid(acc[0][i]);
      const float fg = mta_sigmoid(acc[1][i]);
      const float gg = mta_tanh(acc[2][i]);
      const float og = mta_sigmoid(acc[3][i]);
      c[i] = fmaf(fg, c[i], ig * gg);
      const float h = og * mta_tanh(c[i]);
      const int s = 4 * q + i;
      const int n = n0 + s;
      if (valid[i]) {
        const size_t gb = ((size_t)t * N + n) * G4 + u;
        gates[gb] = ig;
        gates[gb + H] = fg;
        gates[gb + 2 * H] = gg;
        gates[gb + 3 * H] = og;
        const size_t hb = ((size_t)t * N + n) * H + u;
        cseq[hb] = c[i];
        hseq[hb] = h;
      }
      if constexpr (PREC == PREC_F32) {
        h_f[nb][s][(u & 3) * KF + (u >> 2)] = h;
      } else {
        __bf16 hi, lo;
        split_bf16(h, hi, lo);
        h_hi[nb][s][u] = hi;
        if constexpr (PREC == PREC_BF16X3) h_lo[nb][s][u] = lo;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// backward (BPTT, reverse time)
// ---------------------------------------------------------------------------------------------
// Reduction index permutation for dh = dG . W_hh: r' = 8*(u>>1) + 4*(u&1) + g  <->  r = g*H + u.
// A producer lane owns one unit and all 4 gates, so its 4 values for one sequence are
// contiguous in r' (one 8-byte LDS write per sequence), and an MFMA A fragment (8 consecutive
// r') covers units (2p, 2p+1) x gates 0..3.
template <int H>
__device__ __forceinline__ int rperm_to_r(int rp) {
  const int e = rp & 7, p = rp >> 3;
  const int uu = 2 * p + (e >> 2), g = e & 3;
  return g * H + uu;
}

template <int H, int PREC>
__global__ __launch_bounds__((H / 16) * 64) void lstm_bwd_kernel(
    float* gates,                     // (T, N, 4H) in: activated gates; out: dG (pre-activation)
    const float* __restrict__ cseq,   // (T, N, H)
    const float* __restrict__ w_hh,   // (4H, H)
    const float* __restrict__ dH,     // (T, N, H) grad wrt this layer's outputs, or nullptr
    const float* __restrict__ dh_last,// (N, H) grad wrt h_{T-1} only, or nullptr
    int N, int T) {
  constexpr int G4 = 4 * H;
  constexpr int KB = G4 / 32;       // bf16 k-blocks
  constexpr int KF = G4 / 4;        // f32 k-steps
  constexpr int ROWB = G4 + 8;
  constexpr int ROWF = G4 + 4;

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int q = lane >> 4, j = lane & 15;
  const int u = 16 * w + j;
  const int n0 = blockIdx.x * S;

  __shared__ __attribute__((aligned(16))) __bf16 g_hi[2][S][PREC == PREC_F32 ? 8 : ROWB];
  __shared__ __attribute__((aligned(16))) __bf16 g_lo[2][S][PREC == PREC_BF16X3 ? ROWB : 8];
  __shared__ __attribute__((aligned(16))) float g_f[2][S][PREC == PREC_F32 ? ROWF : 4];

  // B fragments: B[r'][k] = W_hh[r(r')][16w + j]
  bf16x8 Bhi[PREC == PREC_F32 ? 1 : KB], Blo[PREC == PREC_BF16X3 ? KB : 1];
  float Bf[PREC == PREC_F32 ? KF : 1];
  if constexpr (PREC == PREC_F32) {
#pragma unroll
    for (int kk = 0; kk < KF; ++kk) Bf[kk] = w_hh[(size_t)(4 * kk + q) * H + u];
  } else {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int r = rperm_to_r<H>(32 * kb + 8 * q + e);
        __bf16 hi, lo;
        split_bf16(w_hh[(size_t)r * H + u], hi, lo);
        Bhi[kb][e] = hi;
        if constexpr (PREC == PREC_BF16X3) Blo[kb][e] = lo;
      }
  }

  bool valid[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) valid[i] = (n0 + 4 * q + i) < N;

  float dc[4] = {0.f, 0.f, 0.f, 0.f};
  float dhr[4] = {0.f, 0.f, 0.f, 0.f};  // recurrent dh from step t+1

  // per-step inputs (prefetched one step ahead)
  float ga[4][4], ct[4], cp[4], dho[4];
  auto load_step = [&](int t, float (&gdst)[4][4], float (&cdst)[4], float (&cpdst)[4], float (&ddst)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + 4 * q + i;
      const size_t hb = ((size_t)t * N + n) * H + u;
      const size_t gb = ((size_t)t * N + n) * G4 + u;
#pragma unroll
      for (int g = 0; g < 4; ++g) gdst[g][i] = valid[i] ? gates[gb + g * H] : 0.f;
      cdst[i] = valid[i] ? cseq[hb] : 0.f;
      cpdst[i] = (valid[i] && t > 0) ? cseq[hb - (size_t)N * H] : 0.f;
      float d = 0.f;
      if (valid[i]) {
        if (dH) d = dH[hb];
        else if (dh_last && t == T - 1) d = dh_last[(size_t)n * H + u];
      }
      ddst[i] = d;
    }
  };
  load_step(T - 1, ga, ct, cp, dho);

  for (int t = T - 1; t >= 0; --t) {
    float g_cur[4][4], c_cur[4], cp_cur[4], dh_cur[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int g = 0; g < 4; ++g) g_cur[g][i] = ga[g][i];
      c_cur[i] = ct[i];
      cp_cur[i] = cp[i];
      dh_cur[i] = dho[i];
    }
    if (t > 0) load_step(t - 1, ga, ct, cp, dho);

    const int buf = t & 1;
    float dG[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float ig = g_cur[0][i], fg = g_cur[1][i], gg = g_cur[2][i], og = g_cur[3][i];
      const float dh = dh_cur[i] + dhr[i];
      const float tc = mta_tanh(c_cur[i]);
      const float d_o = dh * tc * og * (1.f - og);
      const float dcc = fmaf(dh * og, 1.f - tc * tc, dc[i]);
      dG[0][i] = dcc * gg * ig * (1.f - ig);
      dG[1][i] = dcc * cp_cur[i] * fg * (1.f - fg);
      dG[2][i] = dcc * ig * (1.f - gg * gg);
      dG[3][i] = d_o;
      dc[i] = dcc * fg;
      const int s = 4 * q + i;
      const int n = n0 + s;
      if (valid[i]) {
        const size_t gb = ((size_t)t * N + n) * G4 + u;
#pragma unroll
        for (int g = 0; g < 4; ++g) gates[gb + g * H] = dG[g][i];
      }
      if (t > 0) {
        if constexpr (PREC == PREC_F32) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int r = g * H + u;  // identity r' for f32; stored at (r&3)*KF + (r>>2)
            g_f[buf][s][(r & 3) * KF + (r >> 2)] = dG[g][i];
          }
        } else {
          bf16x4 hi4, lo4;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            __bf16 hi, lo;
            split_bf16(dG[g][i], hi, lo);
            hi4[g] = hi;
            lo4[g] = lo;
          }
          const int rp = 8 * (u >> 1) + 4 * (u & 1);
          *reinterpret_cast<bf16x4*>(&g_hi[buf][s][rp]) = hi4;
          if constexpr (PREC == PREC_BF16X3) *reinterpret_cast<bf16x4*>(&g_lo[buf][s][rp]) = lo4;
        }
      }
    }
    if (t == 0) break;
    __syncthreads();

    // ---- dh_{t-1} = dG_t (16 x 4H) . W_hh (4H x 16 cols of this wave) -----------------------
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    if constexpr (PREC == PREC_F32) {
      const float* arow = &g_f[buf][j][q * KF];
#pragma unroll
      for (int kk = 0; kk < KF; kk += 2) {
        acc0 = mfma16x16x4f32(arow[kk], Bf[kk], acc0);
        acc1 = mfma16x16x4f32(arow[kk + 1], Bf[kk + 1], acc1);
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const bf16x8 ahi = *reinterpret_cast<const bf16x8*>(&g_hi[buf][j][32 * kb + 8 * q]);
        if constexpr (PREC == PREC_BF16X3) {
          const bf16x8 alo = *reinterpret_cast<const bf16x8*>(&g_lo[buf][j][32 * kb + 8 * q]);
          acc1 = mfma16x16x32(alo, Bhi[kb], acc1);
          acc1 = mfma16x16x32(ahi, Blo[kb], acc1);
        }
        acc0 = mfma16x16x32(ahi, Bhi[kb], acc0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) dhr[i] = acc0[i] + acc1[i];
  }
}

template <int H, int PREC>
void launch_fwd(const float* x, const float* w_ih, const float* b_ih, const float* b_hh, int fin, const float* gx,
                float* gates, const float* w_hh, float* hseq, float* cseq, int N, int T, hipStream_t st) {
  dim3 grid((N + S - 1) / S), block((H / 16) * 64);
  switch (fin) {
    case 0: lstm_fwd_kernel<H, PREC, 0><<<grid, block, 0, st>>>(x, w_ih, b_ih, b_hh, gx, gates, w_hh, hseq, cseq, N, T); break;
    case 1: lstm_fwd_kernel<H, PREC, 1><<<grid, block, 0, st>>>(x, w_ih, b_ih, b_hh, gx, gates, w_hh, hseq, cseq, N, T); break;
    case 2: lstm_fwd_kernel<H, PREC, 2><<<grid, block, 0, st>>>(x, w_ih, b_ih, b_hh, gx, gates, w_hh, hseq, cseq, N, T); break;
    case 3: lstm_fwd_kernel<H, PREC, 3><<<grid, block, 0, st>>>(x, w_ih, b_ih, b_hh, gx, gates, w_hh, hseq, cseq, N, T); break;
    case 4: lstm_fwd_kernel<H, PREC, 4><<<grid, block, 0, st>>>(x, w_ih, b_ih, b_hh, gx, gates, w_hh, hseq, cseq, N, T); break;
    case 5: lstm_fwd_kernel<H, PREC, 5><<<grid, block, 0, st>>>(x, w_ih, b_ih, b_hh, gx, gates, w_hh, hseq, cseq, N, T); break;
    default: break;
  }
}

template <int H>
void dispatch_fwd(int prec, const float* x, const float* w_ih, const float* b_ih, const float* b_hh, int fin,
                  const float* gx, float* gates, const float* w_hh, float* hseq, float* cseq, int N, int T,
                  hipStream_t st) {
  if (prec == PREC_F32) launch_fwd<H, PREC_F32>(x, w_ih, b_ih, b_hh, fin, gx, gates, w_hh, hseq, cseq, N, T, st);
  else if (prec == PREC_BF16X3) launch_fwd<H, PREC_BF16X3>(x, w_ih, b_ih, b_hh, fin, gx, gates, w_hh, hseq, cseq, N, T, st);
  else launch_fwd<H, PREC_BF16>(x, w_ih, b_ih, b_hh, fin, gx, gates, w_hh, hseq, cseq, N, T, st);
}

template <int H>
void dispatch_bwd(int prec, float* gates, const float* cseq, const float* w_hh, const float* dH,
                  const float* dh_last, int N, int T, hipStream_t st) {
  dim3 grid((N + S - 1) / S), block((H / 16) * 64);
  if (prec == PREC_F32) lstm_bwd_kernel<H, PREC_F32><<<grid, block, 0, st>>>(gates, cseq, w_hh, dH, dh_last, N, T);
  else if (prec == PREC_BF16X3) lstm_bwd_kernel<H, PREC_BF16X3><<<grid, block, 0, st>>>(gates, cseq, w_hh, dH, dh_last, N, T);
  else lstm_bwd_kernel<H, PREC_BF16><<<grid, block, 0, st>>>(gates, cseq, w_hh, dH, dh_last, N, T);
}

}  // namespace

// Returns 0 on success, -1 for an unsupported (H, fin) combination.
extern "C" int mta_lstm_fwd_layer(int H, int prec, const float* x, const float* w_ih, const float* b_ih,
                                  const float* b_hh, int fin, const float* gx, float* gates, const float* w_hh,
                                  float* hseq, float* cseq, int N, int T, hipStream_t st) {
  if (fin < 0 || fin > 5) return -1;
  switch (H) {
    case 32: dispatch_fwd<32>(prec, x, w_ih, b_ih, b_hh, fin, gx, gates, w_hh, hseq, cseq, N, T, st); return 0;
    case 64: dispatch_fwd<64>(prec, x, w_ih, b_ih, b_hh, fin, gx, gates, w_hh, hseq, cseq, N, T, st); return 0;
    case 128: dispatch_fwd<128>(prec, x, w_ih, b_ih, b_hh, fin, gx, gates, w_hh, hseq, cseq, N, T, st); return 0;
    default: return -1;
  }
}

extern "C" int mta_lstm_bwd_layer(int H, int prec, float* gates, const float* cseq, const float* w_hh,
                                  const float* dH, const float* dh_last, int N, int T, hipStream_t st) {
  switch (H) {
    case 32: dispatch_bwd<32>(prec, gates, cseq, w_hh, dH, dh_last, N, T, st); return 0;
    case 64: dispatch_bwd<64>(prec, gates, cseq, w_hh, dH, dh_last, N, T, st); return 0;
    case 128: dispatch_bwd<128>(prec, gates, cseq, w_hh, dH, dh_last, N, T, st); return 0;
    default: return -1;
  }
}
