// Layer-pipelined (wavefront) multi-layer LSTM for MI355X (gfx950): ALL layers in one launch.
//
// The per-layer kernels in lstm.hip run L x T dependent timesteps (L launches of T steps).  Here one
// workgroup runs layer l for one 16-sequence tile, and layer l starts step t as soon as layer l-1 has
// published h^{(l-1)}_t: the critical path becomes ~T + small lag steps instead of L x T
// (reference: the cuDNN multi-layer LSTM of `src/model.py:88-94`; SURVEY.md K1/K2/K3 "diagonal
// (layer, t) wavefront").
//
//   forward : layer 0 fuses its F-wide input projection (as lstm.hip); layers >= 1 compute
//             W_ih x_t with MFMA inside the recurrence (W_ih and W_hh both resident in VGPRs), reading
//             x_t = dropout(h^{(l-1)}_t) that the producer layer stored write-through (sc1) together with
//             the dropout-masked copy (counter-hash mask, common.h), then publishes a per-(layer, tile)
//             progress word.
//   backward: layer l >= 1 also computes dx_t = dG_t W_ih (second MFMA product on the same LDS dG image),
//             applies its input-dropout mask and hands dH^{(l-1)}_t to layer l-1 the same way.
//
// Hand-off protocol (cdna_hip_programming.md Guideline 16, R1 form, placement independent): payload
// stores are sc1 (write-through); every storing wave drains them (s_waitcnt vmcnt(0)) before the
// workgroup barrier after which ONE lane stores the progress word with an agent-scope atomic; the consumer
// polls that word relaxed with s_sleep back-off (bounded: a timeout word is set instead of hanging) and
// reads the payload with sc1 loads only.  Stores stay delayed by one step (lstm.hip), so progress is
// published two steps behind; the consumer keeps a one-step-stale copy of the word so a poll is only
// paid when it actually waits.  All workgroups (L x tiles <= 8 x 16) are co-resident.
//
// Round 6: the forward's default form is stack_fwd_dec (up to 512 padded sequences; ops/lstm.py DEC_MAX_NP): the
// three wave roles hand LDS ring slots to each other through per-wave step counters instead of one workgroup barrier
// per step, and the layer hand-off is data-tagged 8-byte granules instead of payload + progress word.  The backward
// keeps its barrier body (a decoupled backward was slower and not run-to-run stable in bf16; docs/ARCHITECTURE.md),
// with the gradient waves' dH prefetch distance chosen per depth (stack_bwd_body<..., DPF>) and the fused
// weight-gradient chunks of one step split over two workgroups at B = 1.
#include <cstdlib>

#include "common.h"
#if MTA_STAMPS == 2
// diagnostic timeline build: the last weight-gradient workgroup's k-slice starts (0..15), accumulation done (16),
// atomics issued (17)
__device__ unsigned long long mta_stack_tls[18];
#define WG_SLICE_STAMP(k)                                                                                    \
  do {                                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x == gridDim.x - 1 && (k) < 18)                                         \
      mta_stack_tls[(k)] = __builtin_amdgcn_s_memrealtime();                                                 \
  } while (0)
#endif
#include "lstm_wgrad.h"

// diagnostic builds (csrc/tools/lstm_stack_probe.hip): -DMTA_STAMPS=1 per-segment s_memtime sums, -DMTA_STAMPS=2 the
// timeline (s_memtime of every forward workgroup's recurrent wave 0 at entry, after the pre-loop barrier, after step
// T/2 and at the end)
#ifndef MTA_STAMPS
#define MTA_STAMPS 0
#endif
#define STACK_STAMPS (MTA_STAMPS == 1)
#define STACK_TIMELINE (MTA_STAMPS == 2)
#if STACK_TIMELINE
// 100 MHz real-time counter: one clock across XCDs (s_memtime counts per-XCD shader clocks, not aligned)
__device__ unsigned long long mta_stack_tl[2][64][4];
// the backward's last 64 weight-gradient workgroups (by block id: the bottom layer's earliest chunks): entry, chunk
// ready, body done, exit
__device__ unsigned long long mta_stack_tlw[64][4];
#define STACK_TLW(k)                                                                                             \
  do {                                                                                                           \
    const int _r = (int)(gridDim.x - 1 - blockIdx.x);                                                           \
    if (threadIdx.x == 0 && _r < 64) mta_stack_tlw[_r][(k)] = __builtin_amdgcn_s_memrealtime();                 \
  } while (0)
#define STACK_TL(dir, k)                                                                      \
  do {                                                                                        \
    if (threadIdx.x == 0 && blockIdx.x < 64) mta_stack_tl[(dir)][blockIdx.x][(k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define STACK_TL(dir, k) \
  do {                   \
  } while (0)
#define STACK_TLW(k) \
  do {               \
  } while (0)
#endif
// s_sleep units (~64 cycles each) the backward gradient waves wait after a step barrier before their dx MFMA product:
// right after the barrier the recurrent waves run their own MFMA chain on the same SIMDs, and two MFMA streams on one
// SIMD serialise.  4: bwd 98.0 -> 94.5 us at the headline shape; 2: 96, 6: 95.2, 8: 98.2, 12: 104
// (profiles/r4_lstm_knobs.txt).  The dG rows are stored by the recurrent waves (storing them from the gradient waves
// measured slower, profiles/r4_lstm_bwd_dg_negative.txt)
#ifndef DX_DELAY_V  // (diagnostic A/B builds override it)
#define DX_DELAY_V 4
#endif
constexpr int DX_DELAY = DX_DELAY_V;
// static issue priority of the recurrent waves (fwd and bwd) over the input / gradient waves of their SIMD: on
// (fwd 80.0 -> 79.5 us, with DX_DELAY 4 bwd 94.1 us; profiles/r4_lstm_knobs.txt)
#ifndef STACK_PRIO_V  // (diagnostic A/B builds override it)
#define STACK_PRIO_V 1
#endif
constexpr int STACK_PRIO = STACK_PRIO_V;
#if STACK_STAMPS
// Diagnostic build only (csrc/tools/lstm_stack_probe.hip): per-segment s_memtime sums, lane 0 of the first
// wave of each role of block 0 ([direction][role][segment]; role 0 = recurrent, 1 = input / gradient waves).
__device__ unsigned long long mta_stack_stamp_acc[2][3][8];
__device__ int mta_stack_stamp_block[2];  // block whose waves are stamped, per direction (probe sets it)
#define SSTAMP_DECL unsigned long long _ts_prev = 0, _ts_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define SSTAMP(k)                                                                  \
  {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                             \
    const unsigned long long _n = __builtin_amdgcn_s_memtime();                    \
    __builtin_amdgcn_s_waitcnt(0xC07F);                                            \
    if ((k) > 0) _ts_acc[(k)] += _n - _ts_prev;                                    \
    _ts_prev = _n;                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                             \
  }
#define SSTAMP_FLUSH(dir, role, first_wave)                                        \
  if ((int)blockIdx.x == mta_stack_stamp_block[(dir)] && (first_wave) && (threadIdx.x & 63) == 0) \
    for (int _k = 0; _k < 8; ++_k) mta_stack_stamp_acc[(dir)][(role)][_k] = _ts_acc[_k];
#else
#define SSTAMP_DECL
#define SSTAMP(k)
#define SSTAMP_FLUSH(dir, role, first_wave)
#endif

namespace {

constexpr int S = 16;
constexpr int STASH = 5;
constexpr int MAXL = 8;
constexpr unsigned SPIN_LIMIT = 1u << 21;  // default poll bound (env MTA_LSTM_SPIN_LIMIT overrides: fault tests)
constexpr int FLAG_STRIDE = 32;
constexpr int TRS = 20;  // row stride (floats) of the per-wave 16 x 16 transpose scratch (conflict-free writes)
// progress words are E << eshift | steps: eshift = epoch_shift(T) >= 12 bits (long sequences take more step bits;
// the flag buffer a launch uses is keyed by its shift on the host, ops/lstm.py _stack_flags)
constexpr int MIN_EPOCH_SHIFT = 12, MAX_EPOCH_SHIFT = 22;
inline int epoch_shift(int T) {
  int s = MIN_EPOCH_SHIFT;
  while (s < MAX_EPOCH_SHIFT && (1 << s) <= T + 8) ++s;
  return s;
}

__device__ __forceinline__ size_t stash_index(int t, int tile, int ntiles, int w, int nw, int lane) {
  // component k of a lane at + 64 k: every stash store / load instruction covers 1 KB contiguous
  return (((size_t)t * ntiles + tile) * nw + w) * (64 * STASH) + lane;
}

__device__ __forceinline__ void store_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte write-through store (the dG rows the fused weight-gradient workgroups read); one vector-memory op.
// The s_nop covers the >8-byte store-data hazard (the hazard recognizer does not see into inline asm: a
// VALU write to the data VGPRs right after the store would corrupt what it stores).
__device__ __forceinline__ void store_sc1_x4(float* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}

// Control words (one 128-byte line each) after the three progress regions.
constexpr int CTL_TIMEOUT = 0, CTL_FWD_EPOCH = 32, CTL_FWD_DONE = 64, CTL_BWD_EPOCH = 96, CTL_BWD_DONE = 128;
constexpr int CTL_WORDS = 160;

// XCD-local hand-off fast path.  Producer and consumer of a layer hand-off are tile i of adjacent layers, block ids
// equal modulo 8, i.e. normally on one XCD (blocks are dealt round-robin over the XCDs).  Correctness must not
// depend on that (cdna_hip_programming.md Guideline 16), so every workgroup publishes the XCC id it runs on
// (HW_REG_XCC_ID, epoch-tagged, in the table in front of the control words) and a producer uses PLAIN stores and a
// plain progress store -- which stay in the XCD's L2, where the consumer's sc1 (L1-bypassing, L2-served) loads and
// polls find them -- only when its consumer reported the SAME XCC; otherwise the write-through (sc1) form, whose
// lines the fabric serves to any XCD.  Same-XCD sc1 stores drop the L2 line (MI355X_MICROARCH.md § visibility),
// so the fast path saves the fabric round trip on every hand-off.  MTA_LSTM_XCD_LOCAL=0 disables it.
__device__ __forceinline__ unsigned my_xcc() {
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;  // hwreg(HW_REG_XCC_ID, 0, 4)
}
__device__ __forceinline__ void publish_xcc(unsigned* slot, unsigned epoch) {
  __hip_atomic_store(slot, (epoch << 4) | my_xcc(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// whether the workgroup that publishes into `slot` for `epoch` runs on this XCC (bounded wait: false on give-up)
__device__ __forceinline__ bool partner_local(const unsigned* slot, unsigned epoch, unsigned limit) {
  for (unsigned spins = 0; spins <= limit; ++spins) {
    const unsigned v = __hip_atomic_load(const_cast<unsigned*>(slot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((v >> 4) == (epoch & 0x0FFFFFFFu)) return (v & 15u) == my_xcc();
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}
__device__ __forceinline__ void store_plain_x4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void store_flag(unsigned* flag, unsigned v, bool local) {
  if (local) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // plain store: stays in L2
  else __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned read_epoch_base(unsigned* ctl, int which, int eshift) {
  return __hip_atomic_load(ctl + which, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) << eshift;
}
// every workgroup arrives once after its work; the last one re-arms the counter and advances the epoch
// (every workgroup read the epoch before arriving, so no launch sees a torn value)
__device__ __forceinline__ bool finish_launch(unsigned* ctl, int epoch_word, int done_word, unsigned base,
                                              int eshift) {
  __syncthreads();
  if (threadIdx.x != 0) return false;
  const unsigned prev = __hip_atomic_fetch_add(ctl + done_word, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (prev != gridDim.x - 1) return false;
  __hip_atomic_store(ctl + done_word, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(ctl + epoch_word, (base >> eshift) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// Progress words are never reset: a launch reads its epoch E (control word, advanced by the launch's last
// workgroup) and publishes (E << eshift) + steps, so a stale word of an earlier launch always compares below
// (wrap-safe signed difference, T + 8 < 2^eshift).  No memset node per launch.
__device__ __forceinline__ bool reached(unsigned seen, unsigned need) { return (int)(seen - need) >= 0; }

// wait until *flag reaches need (relaxed agent-scope polls); returns the value seen.  A wait that exceeds
// `limit` polls gives up (so the grid always drains) and counts itself in the timeout word, which the host
// checks (ops.lstm.check_pipeline_health: the trainer raises at epoch end, bench.py at the end of the run).
__device__ __forceinline__ unsigned wait_progress(unsigned* flag, unsigned need, unsigned seen, unsigned* tmo,
                                                  unsigned limit) {
  unsigned spins = 0;
  while (!reached(seen, need)) {
    __builtin_amdgcn_s_sleep(1);
    seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (++spins > limit) {
      __hip_atomic_fetch_add(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      seen = need;  // give up waiting (results are garbage: the host raises on the non-zero timeout count)
    }
  }
  // every payload load after this point is sc1 (L1 bypass): only keep the compiler from hoisting them
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return seen;
}

// wait_progress for a workgroup that waits many steps (the fused weight-gradient chunks: up to T steps, ~240 of
// them per launch at B = 1, L = 2): the sleep between polls grows with the distance still to go (a step is ~1 us,
// s_sleep(127) ~4 us), so the pollers do not keep the progress words' lines busy for the pipeline's own hand-offs.
__device__ __forceinline__ unsigned wait_progress_far(unsigned* flag, unsigned need, unsigned seen, unsigned* tmo,
                                                      unsigned limit) {
  unsigned spins = 0;
  seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (!reached(seen, need)) {
    const unsigned gap = need - seen;  // steps still to go (a previous launch's value: a huge gap)
    if (gap > 8) __builtin_amdgcn_s_sleep(127);
    else if (gap > 2) __builtin_amdgcn_s_sleep(24);
    else __builtin_amdgcn_s_sleep(1);
    seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (++spins > limit) {
      __hip_atomic_fetch_add(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      seen = need;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return seen;
}

// 16 bytes of handed-off data as two 8-byte agent-scope atomic loads (global_load_dwordx2 ... sc1:
// L1-bypassing, the consumer form of the sc1 hand-off)
__device__ __forceinline__ float4 load_sc1(const float* base, size_t elem) {
  unsigned long long* p = reinterpret_cast<unsigned long long*>(const_cast<float*>(base) + elem);
  const unsigned long long a = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long b = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  float4 o;
  o.x = __builtin_bit_cast(float, (unsigned)a);
  o.y = __builtin_bit_cast(float, (unsigned)(a >> 32));
  o.z = __builtin_bit_cast(float, (unsigned)b);
  o.w = __builtin_bit_cast(float, (unsigned)(b >> 32));
  return o;
}

struct StackFwdArgs {
  const float* x;  // layer-0 input (N, T, FIN0), batch-first
  const float* w_ih[MAXL];
  const float* w_hh[MAXL];
  const float* b_ih[MAXL];
  const float* b_hh[MAXL];
  float* hseq[MAXL];    // (T, Np, H) outputs of every layer
  float* xdrop[MAXL];   // xdrop[l] (l >= 1): dropout(h^{(l-1)}), the input of layer l (null: no dropout)
  uint32_t* mask[MAXL]; // mask[l] (with xdrop[l]): keep bytes of that dropout, (T, ntiles, S, H/4) words
                        // (stack_keep_index: byte e of word (t, tile, s, c) = unit 4c+e of sequence s), read by the backward
  float* stash[MAXL];   // BPTT stash per layer (null: inference)
  const uint64_t* seeds;  // [MAXL]: seed of the dropout applied to layer l's input
  float drop_p;
  unsigned* flags;      // [MAXL][tr8] progress words (epoch-stamped, never reset)
  unsigned* timeout;
  unsigned* ctl;
  unsigned* xcc;        // [MAXL][tr8] epoch-tagged XCC ids of this direction's workgroups
  int xcd_local;        // XCD-local hand-off fast path enabled
  unsigned spin_limit;
  int N, Np, T, L, ntiles, tr8, eshift;
  // in-kernel batch gather (gather != 0): layer 0 reads x through the device permutation, copy_blocks extra
  // workgroups at the end of the grid copy the batch rows into the static buffers (the decoder and the backward
  // read those) on otherwise idle CUs while the recurrence runs, the last workgroup advances the cursor: no
  // separate gather launch per training step
  int gather, copy_blocks, main_blocks;
  MtaBatchGather g;
  // decoupled form (stack_fwd_dec): gran[l] (l >= 1) = layer l's input as tagged granules (T, Np, H) x 8 bytes
  unsigned long long* gran[MAXL];
  int dec;  // 1: stack_fwd_dec (the default), 0: the barrier form (MTA_LSTM_DEC=0, A/B)
};

// Forward workgroup = 3 x (H/16) waves in three roles (one wave of each role per SIMD):
//   RECURRENT waves [0, NW): W_hh in VGPRs, h through LDS, one barrier per step -- and NO global memory
//     operation inside the time loop: h_t (fp32) and the BPTT stash of step t go to LDS staging slots.
//   INPUT waves [NW, 2 NW): one step ahead they wait for / load the layer input and compute the gate
//     pre-activations gx_{t+1} = bias + W_ih x_{t+1} (fused F-wide dot products for layer 0, MFMA for layers
//     >= 1) into a double-buffered LDS slot (hand-off latency, progress polls and the input product off the
//     recurrent path).
//   STORE waves [2 NW, 3 NW): during step t they write out step t-1 from the staging slots: h (write-through when
//     a layer above consumes it), the dropout-masked copy for the next layer with its keep bytes (pair hash,
//     common.h), the stash; they drain the write-through stores and publish the layer's progress word.
// r2 stamp probe: store issue + vmcnt drain were ~700 of ~2600 cycles of a recurrent step when the recurrent
// waves issued the stores themselves.  All roles execute the same barriers (pre-loop, one per step, final).
// MFMA operand element / fragment types of a precision mode (PREC_F16X2: fp16, the others: bf16)
template <int PREC>
struct OpT {
  using E = __bf16;
  using V8 = bf16x8;
};
template <>
struct OpT<PREC_F16X2> {
  using E = _Float16;
  using V8 = f16x8;
};
// the weight operand has a lo half (bf16x3: hi + lo of both operands; f16x2: hi + lo of the weight only)
template <int PREC>
constexpr bool kWeightLo = PREC == PREC_BF16X3 || PREC == PREC_F16X2;
// MFMA passes per k-block: bf16x3 lo*Whi + hi*Wlo + hi*Whi; f16x2 a*Wlo + a*Whi; bf16 a*Whi
template <int PREC>
constexpr int kPasses = PREC == PREC_BF16X3 ? 3 : PREC == PREC_F16X2 ? 2 : 1;

template <int H, int PREC>
struct FwdSmem {
  static constexpr int ROWB = H + 8, ROWF = H + 4;
  using E = typename OpT<PREC>::E;
  float4 gxs[2][S][H];  // gate pre-activations (i, f, g, o) per (sequence, unit)
  E h_hi[2][S][PREC == PREC_F32 ? 8 : ROWB];
  __bf16 h_lo[2][S][PREC == PREC_BF16X3 ? ROWB : 8];
  float h_f[2][S][PREC == PREC_F32 ? ROWF : 4];
  // layers >= 1: the layer input x_t (slot t & 1) in the MFMA A-operand layout, filled a quarter per input wave
  E x_hi[2][S][PREC == PREC_F32 ? 8 : ROWB];
  __bf16 x_lo[2][S][PREC == PREC_BF16X3 ? ROWB : 8];
  float x_f[2][S][PREC == PREC_F32 ? ROWF : 4];
  float hout[3][S][ROWF];              // h_t in fp32, natural unit order (slot t % 3), for the store waves
  float4 st[3][H / 16][STASH][64];     // BPTT stash of step t (slot t % 3), per recurrent wave, lane-major
};

// keep bits of the forward dropout on layer l's input (store layout: one word per (row, 4 units), byte e = unit
// 4 c + e): row = t * Np + n, pair hash over column pairs (the backward reads the same words)
__device__ __forceinline__ uint32_t stack_keep_word(uint32_t pseed, uint32_t row, int unit4, float p) {
  const uint32_t h0 = mta_pair_hash(pseed, row, mta_pair_col((uint32_t)unit4 >> 1));
  const uint32_t h1 = mta_pair_hash(pseed, row, mta_pair_col(((uint32_t)unit4 >> 1) + 1));
  return (mta_pair_keep(h0, 0, p) ? 1u : 0u) | (mta_pair_keep(h0, 1, p) ? 1u << 8 : 0u) |
         (mta_pair_keep(h1, 0, p) ? 1u << 16 : 0u) | (mta_pair_keep(h1, 1, p) ? 1u << 24 : 0u);
}
__device__ __forceinline__ size_t stack_keep_index(int t, int tile, int ntiles, int s, int H, int unit4) {
  return (((size_t)t * ntiles + tile) * S + s) * (H / 4) + unit4 / 4;
}

template <int H, int PREC, int FIN0, bool FIRST>
__device__ __forceinline__ void stack_fwd_body(const StackFwdArgs& a, const int layer, const int tile,
                                               FwdSmem<H, PREC>& sm, const unsigned base) {
  constexpr int NW = H / 16;
  constexpr int KB = H / 32;
  constexpr int KF = H / 4;
  constexpr int XR = H / 16;  // float4 of a layer input row per lane (bf16: 2 per k-block; f32: KF/4)
  constexpr int ROWB = H + 8;
  constexpr int ROWF = H + 4;

  using E = typename OpT<PREC>::E;
  using V8 = typename OpT<PREC>::V8;
  const bool last = layer == a.L - 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int role = wave / NW;  // 0 recurrent, 1 input, 2 store
  const bool input_wave = role == 1;
  const int w = wave - role * NW;
  const int q = lane >> 4, j = lane & 15;
  const int u = 16 * w + j;
  const int n0 = tile * S;
  const int N = a.N, Np = a.Np, T = a.T;

  auto& gxs = sm.gxs;
  auto& h_hi = sm.h_hi;
  auto& h_lo = sm.h_lo;
  auto& h_f = sm.h_f;

  float bias[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bias[g] = a.b_ih[layer][g * H + u] + a.b_hh[layer][g * H + u];

  if (role == 2) {
    // =========================== store waves ===========================
    float* hseq = a.hseq[layer];
    float4* stash = reinterpret_cast<float4*>(a.stash[layer]);
    float* xout = last ? nullptr : a.xdrop[layer + 1];
    uint32_t* mout = xout ? a.mask[layer + 1] : nullptr;
    const uint32_t pseed = mout ? mta_pair_seed(a.seeds[layer + 1]) : 0;
    const float keep_scale = 1.0f / (1.0f - a.drop_p);
    unsigned* my_flag = a.flags + FLAG_STRIDE * (layer * a.tr8 + tile);
    const int ts = lane >> 2, tc = 4 * (lane & 3), unit4 = 16 * w + tc;
    const unsigned E = base >> a.eshift;
    if (w == 0 && lane == 0) publish_xcc(a.xcc + layer * a.tr8 + tile, E);
    // every store wave learns for itself whether its consumer (tile `tile` of layer + 1) shares this XCD's L2
    const bool local = a.xcd_local && !last && partner_local(a.xcc + (layer + 1) * a.tr8 + tile, E, 1u << 14);
    // step t from staging slot t & 1: hand-offs first (h, masked h), then keep word and stash (issue order per
    // interval, the loop-head vmcnt counts below depend on it)
    auto store_step = [&](int t) {
      const int slot = t % 3;
      const float4 hv = *reinterpret_cast<const float4*>(&sm.hout[slot][ts][unit4]);
      const size_t o = ((size_t)t * Np + n0 + ts) * H + unit4;
      if (last || local) store_plain_x4(hseq + o, f32x4{hv.x, hv.y, hv.z, hv.w});  // last: consumed after the kernel
      else store_sc1_x4(hseq + o, f32x4{hv.x, hv.y, hv.z, hv.w});
      if (xout) {
        const uint32_t kw = stack_keep_word(pseed, (uint32_t)(t * Np + n0 + ts), unit4, a.drop_p);
        const f32x4 xv{hv.x * ((kw & 0xFFu) ? keep_scale : 0.f), hv.y * ((kw & 0xFF00u) ? keep_scale : 0.f),
                       hv.z * ((kw & 0xFF0000u) ? keep_scale : 0.f), hv.w * ((kw & 0xFF000000u) ? keep_scale : 0.f)};
        if (local) store_plain_x4(xout + o, xv);
        else store_sc1_x4(xout + o, xv);
        mout[stack_keep_index(t, tile, a.ntiles, ts, H, unit4)] = kw;
      }
      if (stash) {
#pragma unroll
        for (int k = 0; k < STASH; ++k)
          stash[stash_index(t, tile, a.ntiles, w, NW, lane) + 64 * k] = sm.st[slot][w][k][lane];
      }
    };
    __syncthreads();  // P0
    __syncthreads();  // P1 (pre-loop)
    SSTAMP_DECL
    // interval t (between barriers B(t-1) and B(t), while the recurrent waves run step t) writes out step t-2:
    // the recurrent waves stage step t-1 in its slot during step t (LDS writes beside their MFMA chain)
    for (int t = 0; t < T; ++t) {
      SSTAMP(0)
      // drain the hand-offs issued two intervals ago (step t-4); newer: that interval's [keep word, stash] and
      // the previous interval's [h, masked h, keep word, stash].  Immediates: branch on the uniform layout.
      if (t >= 4) {
        if (xout) {
          if (stash) mta_wait_vmcnt<(1 + STASH) + (3 + STASH)>();
          else mta_wait_vmcnt<1 + 3>();
        } else {
          if (stash) mta_wait_vmcnt<STASH + (1 + STASH)>();
          else mta_wait_vmcnt<1>();
        }
      }
      // progress: the hand-offs of step t-5 were drained by every store wave's wait at the top of interval
      // t-1, before the barrier that ended it
      if (!last && t >= 5 && wave == 2 * NW && lane == 0) store_flag(my_flag, base + (unsigned)(t - 4), local);
      SSTAMP(1)
      if (t >= 2) store_step(t - 2);
      SSTAMP(2)
      __syncthreads();
      SSTAMP(3)
    }
    SSTAMP_FLUSH(0, 1, w == 0)
    if (T >= 2) store_step(T - 2);
    __syncthreads();  // F1: step T-1 staged
    store_step(T - 1);
    mta_wait_vmem();
    __syncthreads();  // F2 (final)
    if (!last && wave == 2 * NW && lane == 0) store_flag(my_flag, base + (unsigned)T, local);
    return;
  }

  if (input_wave) {
    // =========================== input waves ===========================
    const float* w_ih = a.w_ih[layer];
    const float* xin = FIRST ? nullptr : (a.xdrop[layer] ? a.xdrop[layer] : a.hseq[layer - 1]);
    unsigned* in_flag = a.flags + FLAG_STRIDE * (FIRST ? 0 : (layer - 1) * a.tr8 + tile);
    constexpr int XKB = FIRST ? 1 : KB, XKF = FIRST ? 1 : KF;
    V8 Xhi[4][PREC == PREC_F32 ? 1 : XKB], Xlo[4][kWeightLo<PREC> ? XKB : 1];
    float Xf[4][PREC == PREC_F32 ? XKF : 1];
    float wi[4][FIRST ? FIN0 : 1];
    if constexpr (FIRST) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int f = 0; f < FIN0; ++f) wi[g][f] = w_ih[(g * H + u) * FIN0 + f];
    } else if constexpr (PREC == PREC_F32) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int kk = 0; kk < KF; ++kk) Xf[g][kk] = w_ih[(size_t)(g * H + u) * H + KF * q + kk];
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            E hi, lo;
            split_bf16(w_ih[(size_t)(g * H + u) * H + 32 * kb + 8 * q + e], hi, lo);
            Xhi[g][kb][e] = hi;
            if constexpr (kWeightLo<PREC>) Xlo[g][kb][e] = lo;
          }
    }
    int nrow[4];
    float nmask[4];
    const float* xbase[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + 4 * q + i;
      nrow[i] = n < N ? n : N - 1;
      nmask[i] = n < N ? 1.f : 0.f;
      if constexpr (FIRST) {
        if (a.gather) {
          // sequence n = stock (n % K) of batch window b = n / K, read where the dataset holds it
          const int K = N / a.g.B, b = nrow[i] / K, s = nrow[i] - b * K;
          const int w = a.g.perm[a.g.cursor[0] * a.g.B + b];
          xbase[i] = a.g.src[0] + (size_t)w * a.g.row[0] + (size_t)s * T * FIN0;
        } else {
          xbase[i] = a.x + (size_t)nrow[i] * T * FIN0;
        }
      }
    }
    // Layer inputs are prefetched THREE steps ahead into two register sets (step s in set s & 1): a
    // write-through hand-off is read from beyond L2 (sc1 stores drop the line), ~1-2 us, i.e. more than the one
    // interval the single-set form gave it (layer >= 1 input waves waited on it every step, r2 stamp probe).
    struct XBuf {
      float x0[4][FIRST ? FIN0 : 1];
      float4 xr[FIRST ? 1 : XR];
    };
    XBuf xbA, xbB;
    unsigned seen = base;
    auto load_input = [&](int t, XBuf& xb) {
      if constexpr (FIRST) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float* xs = xbase[i] + (size_t)t * FIN0;
#pragma unroll
          for (int f = 0; f < FIN0; ++f) xb.x0[i][f] = xs[f];
        }
      } else {
        // poll only when the last value seen does not cover step t (polling every step from every
        // consumer wave measured slower: the progress words share cache lines across tiles)
        seen = wait_progress(in_flag, base + (unsigned)(t + 1), seen, a.timeout, a.spin_limit);
        const size_t row = (size_t)t * Np + n0 + j;
#pragma unroll
        for (int v = 0; v < XR; ++v) {
          // bf16: float4 v covers k = 32 (v/2) + 8 q + 4 (v&1) .. +4;  f32: k = KF q + 4 v .. +4
          const int k = PREC == PREC_F32 ? KF * q + 4 * v : 32 * (v >> 1) + 8 * q + 4 * (v & 1);
          xb.xr[v] = load_sc1(xin, row * H + k);
        }
      }
    };
    auto compute_gx = [&](int slot, const XBuf& xb) {
      const auto& xin0 = xb.x0;
      const auto& xr = xb.xr;
      f32x4 acc[4];
      if constexpr (FIRST) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float sacc = bias[g];
#pragma unroll
            for (int f = 0; f < FIN0; ++f) sacc = fmaf(xin0[i][f] * nmask[i], wi[g][f], sacc);
            acc[g][i] = sacc;
          }
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = f32x4{bias[g], bias[g], bias[g], bias[g]};
        if constexpr (PREC == PREC_F32) {
#pragma unroll
          for (int kk = 0; kk < KF; ++kk) {
            const float4 v4 = xr[kk >> 2];
            const float av = (kk & 3) == 0 ? v4.x : (kk & 3) == 1 ? v4.y : (kk & 3) == 2 ? v4.z : v4.w;
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[g] = mfma16x16x4f32(av, Xf[g][kk], acc[g]);
          }
        } else {
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
            const float4 v0 = xr[2 * kb], v1 = xr[2 * kb + 1];
            const float xv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
            V8 ahi, alo;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              E hi, lo;
              split_bf16(xv[e], hi, lo);
              ahi[e] = hi;
              alo[e] = lo;
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              if constexpr (PREC == PREC_BF16X3) {
                acc[g] = mfma16x16x32(alo, Xhi[g][kb], acc[g]);
                acc[g] = mfma16x16x32(ahi, Xlo[g][kb], acc[g]);
              }
              if constexpr (PREC == PREC_F16X2) acc[g] = mfma16x16x32(ahi, Xlo[g][kb], acc[g]);
              acc[g] = mfma16x16x32(ahi, Xhi[g][kb], acc[g]);
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) gxs[slot][4 * q + i][u] = make_float4(acc[0][i], acc[1][i], acc[2][i], acc[3][i]);
    };
    SSTAMP_DECL
    if constexpr (FIRST) {
      load_input(0, xbA);
      compute_gx(0, xbA);
      if (T > 1) load_input(1, xbB);
      if (T > 2) load_input(2, xbA);
      __syncthreads();  // P0
      __syncthreads();  // P1 (pre-loop): gx_0 ready
      // interval t computes gx_{t+1} from set (t+1) & 1 and refills that set with x_{t+3}; unrolled by two so
      // the sets are static registers
      auto interval = [&](int t, XBuf& xb) {
        SSTAMP(0)
        if (t + 1 < T) {
          SSTAMP(1)
          compute_gx((t + 1) & 1, xb);          // x_{t+1}, loaded two intervals ago
          SSTAMP(2)
          if (t + 3 < T) load_input(t + 3, xb);
          SSTAMP(3)
        }
        __syncthreads();
        SSTAMP(4)
      };
      for (int t = 0; t < T; t += 2) {
        interval(t, xbB);
        if (t + 1 < T) interval(t + 1, xbA);
      }
    } else {
      // Layers >= 1: every input wave loads a QUARTER of x_t (units [16w, 16w + 16) of the 16 sequences: one
      // float4 per lane) and writes it split into the shared LDS image; every wave then reads its MFMA A
      // fragments from the image.  4x fewer hand-off loads and splits per wave than each wave loading all of
      // x_t (r3 stamps: that input work set the layer-1 pace).  x_s is polled + loaded 4 intervals ahead into
      // register set s & 1, written into image slot s & 1 two intervals ahead, consumed one interval ahead.
      const int ls = lane >> 2, lu = 16 * w + 4 * (lane & 3);
      float4 xqA = make_float4(0.f, 0.f, 0.f, 0.f), xqB = xqA;
      unsigned seen = base;
      auto load_q = [&](int t, float4& xq) {
        seen = wait_progress(in_flag, base + (unsigned)(t + 1), seen, a.timeout, a.spin_limit);
        xq = load_sc1(xin, ((size_t)t * Np + n0 + ls) * H + lu);
      };
      auto write_q = [&](int t, const float4& xq) {
        const int slot = t & 1;
        if constexpr (PREC == PREC_F32) {
          *reinterpret_cast<float4*>(&sm.x_f[slot][ls][lu]) = xq;
        } else {
          const float xv[4] = {xq.x, xq.y, xq.z, xq.w};
          if constexpr (PREC == PREC_F16X2) {  // one fp16 per element (the activation operand is not split)
            typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
            f16x4_t v4;
#pragma unroll
            for (int e = 0; e < 4; ++e) v4[e] = (_Float16)xv[e];
            *reinterpret_cast<f16x4_t*>(&sm.x_hi[slot][ls][lu]) = v4;
          } else {
            bf16x4 hi4, lo4;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              __bf16 hi, lo;
              split_bf16(xv[e], hi, lo);
              hi4[e] = hi;
              lo4[e] = lo;
            }
            *reinterpret_cast<bf16x4*>(&sm.x_hi[slot][ls][lu]) = hi4;
            if constexpr (PREC == PREC_BF16X3) *reinterpret_cast<bf16x4*>(&sm.x_lo[slot][ls][lu]) = lo4;
          }
        }
      };
      auto compute_gx_img = [&](int t) {  // gx_t from image slot t & 1 into gxs slot t & 1
        const int slot = t & 1;
        f32x4 acc[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = f32x4{bias[g], bias[g], bias[g], bias[g]};
        if constexpr (PREC == PREC_F32) {
          const float* xr = &sm.x_f[slot][j][KF * q];
#pragma unroll
          for (int kk = 0; kk < KF; ++kk) {
            const float av = xr[kk];
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[g] = mfma16x16x4f32(av, Xf[g][kk], acc[g]);
          }
        } else {
          V8 ahi[KB];
          bf16x8 alo[PREC == PREC_BF16X3 ? KB : 1];
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
            ahi[kb] = *reinterpret_cast<const V8*>(&sm.x_hi[slot][j][32 * kb + 8 * q]);
            if constexpr (PREC == PREC_BF16X3) alo[kb] = *reinterpret_cast<const bf16x8*>(&sm.x_lo[slot][j][32 * kb + 8 * q]);
          }
#pragma unroll
          for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              if constexpr (PREC == PREC_BF16X3) {
                acc[g] = mfma16x16x32(alo[kb], Xhi[g][kb], acc[g]);
                acc[g] = mfma16x16x32(ahi[kb], Xlo[g][kb], acc[g]);
              }
              if constexpr (PREC == PREC_F16X2) acc[g] = mfma16x16x32(ahi[kb], Xlo[g][kb], acc[g]);
              acc[g] = mfma16x16x32(ahi[kb], Xhi[g][kb], acc[g]);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) gxs[slot][4 * q + i][u] = make_float4(acc[0][i], acc[1][i], acc[2][i], acc[3][i]);
      };
      load_q(0, xqA);
      if (T > 1) load_q(1, xqB);
      write_q(0, xqA);
      if (T > 1) write_q(1, xqB);
      if (T > 2) load_q(2, xqA);
      if (T > 3) load_q(3, xqB);
      __syncthreads();  // P0: image slots 0 and 1 complete
      compute_gx_img(0);
      __syncthreads();  // P1 (pre-loop): gx_0 ready
      // interval t: x_{t+2} (set t & 1) -> image slot t & 1 (x_t there was consumed in interval t-1); gx_{t+1}
      // from slot (t+1) & 1; refill set t & 1 with x_{t+4}
      auto interval = [&](int t, float4& xq) {
        SSTAMP(0)
        {
          if (t + 2 < T) write_q(t + 2, xq);
          SSTAMP(1)
          if (t + 1 < T) compute_gx_img(t + 1);
          SSTAMP(2)
          if (t + 4 < T) load_q(t + 4, xq);
          SSTAMP(3)
        }
        __syncthreads();
        SSTAMP(4)
      };
      for (int t = 0; t < T; t += 2) {
        interval(t, xqA);
        if (t + 1 < T) interval(t + 1, xqB);
      }
    }
    SSTAMP_FLUSH(0, 2, w == 0)
    __syncthreads();  // F1
    __syncthreads();  // F2 (final; the store waves publish after it)
    return;
  }

  // =========================== recurrent waves ===========================
  STACK_TL(0, 0);
  if (__builtin_amdgcn_readfirstlane(wave) < NW) __builtin_amdgcn_s_setprio(STACK_PRIO);
  const float* w_hh = a.w_hh[layer];
  const bool stash = a.stash[layer] != nullptr;

  V8 Bhi[4][PREC == PREC_F32 ? 1 : KB], Blo[4][kWeightLo<PREC> ? KB : 1];
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
          E hi, lo;
          split_bf16(w_hh[(size_t)(g * H + u) * H + 32 * kb + 8 * q + e], hi, lo);
          Bhi[g][kb][e] = hi;
          if constexpr (kWeightLo<PREC>) Blo[g][kb][e] = lo;
        }
  }
  if constexpr (PREC == PREC_F32) {
    for (int idx = threadIdx.x; idx < S * ROWF; idx += NW * 64) (&h_f[0][0][0])[idx] = 0.f;
  } else {
    for (int idx = threadIdx.x; idx < S * ROWB; idx += NW * 64) (&h_hi[0][0][0])[idx] = (E)0.f;
    if constexpr (PREC == PREC_BF16X3)
      for (int idx = threadIdx.x; idx < S * ROWB; idx += NW * 64) (&h_lo[0][0][0])[idx] = (__bf16)0.f;
  }
  __syncthreads();  // P0
  __syncthreads();  // P1 (pre-loop)
  STACK_TL(0, 1);

  float c[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 pgi, pgf, pgg, pgo, pcc;
  float h[4];
  // step t-1's fp32 h and BPTT stash go to staging slot (t-1) % 3 at the top of step t, where their LDS transfer
  // overlaps this step's MFMA chain (issued before the barrier they stalled the step ~600 cycles, r3 stamps)
  auto stage = [&](int t) {
    const int slot = t % 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) sm.hout[slot][4 * q + i][u] = h[i];
    if (stash) {
      sm.st[slot][w][0][lane] = make_float4(pgi[0], pgi[1], pgi[2], pgi[3]);
      sm.st[slot][w][1][lane] = make_float4(pgf[0], pgf[1], pgf[2], pgf[3]);
      sm.st[slot][w][2][lane] = make_float4(pgg[0], pgg[1], pgg[2], pgg[3]);
      sm.st[slot][w][3][lane] = make_float4(pgo[0], pgo[1], pgo[2], pgo[3]);
      sm.st[slot][w][4][lane] = make_float4(pcc[0], pcc[1], pcc[2], pcc[3]);
    }
  };
  SSTAMP_DECL
  for (int t = 0; t < T; ++t) {
    SSTAMP(0)
    const int cur = t & 1;
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 v = gxs[cur][4 * q + i][u];
      acc[0][i] = v.x;
      acc[1][i] = v.y;
      acc[2][i] = v.z;
      acc[3][i] = v.w;
    }
    SSTAMP(1)
    if constexpr (PREC == PREC_F32) {
      if (t > 0) stage(t - 1);
      const float* hrow = &h_f[cur][j][q * KF];
#pragma unroll
      for (int kk = 0; kk < KF; ++kk) {
        const float av = hrow[kk];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = mfma16x16x4f32(av, Bf[g][kk], acc[g]);
      }
    } else {
      // every A fragment first, then 4 independent MFMA chains (one per gate): per k-block [lo x hi, hi x lo,]
      // hi x hi
      V8 ahi[KB];
      bf16x8 alo[PREC == PREC_BF16X3 ? KB : 1];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        ahi[kb] = *reinterpret_cast<const V8*>(&h_hi[cur][j][32 * kb + 8 * q]);
        if constexpr (PREC == PREC_BF16X3) alo[kb] = *reinterpret_cast<const bf16x8*>(&h_lo[cur][j][32 * kb + 8 * q]);
      }
      if (t > 0) stage(t - 1);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
        for (int sg = 0; sg < kPasses<PREC>; ++sg) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            if constexpr (PREC == PREC_BF16X3) {
              if (sg == 0) acc[g] = mfma16x16x32(alo[kb], Bhi[g][kb], acc[g]);
              else if (sg == 1) acc[g] = mfma16x16x32(ahi[kb], Blo[g][kb], acc[g]);
              else acc[g] = mfma16x16x32(ahi[kb], Bhi[g][kb], acc[g]);
            } else if constexpr (PREC == PREC_F16X2) {
              if (sg == 0) acc[g] = mfma16x16x32(ahi[kb], Blo[g][kb], acc[g]);
              else acc[g] = mfma16x16x32(ahi[kb], Bhi[g][kb], acc[g]);
            } else {
              acc[g] = mfma16x16x32(ahi[kb], Bhi[g][kb], acc[g]);
            }
          }
        }
      }
    }
    SSTAMP(2)
    const int nb = (t + 1) & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pgi[i] = mta_sigmoid(acc[0][i]);
      pgf[i] = mta_sigmoid(acc[1][i]);
      pgg[i] = mta_tanh(acc[2][i]);
      pgo[i] = mta_sigmoid(acc[3][i]);
      c[i] = fmaf(pgf[i], c[i], pgi[i] * pgg[i]);
      pcc[i] = c[i];
      h[i] = pgo[i] * mta_tanh(c[i]);
    }
    SSTAMP(3)
    // next step's A operand first (the critical path), then the staging slots of the store waves
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s4 = 4 * q + i;
      if constexpr (PREC == PREC_F32) {
        h_f[nb][s4][(u & 3) * KF + (u >> 2)] = h[i];
      } else {
        if constexpr (PREC == PREC_F16X2) {
          h_hi[nb][s4][u] = (_Float16)h[i];
        } else {
          __bf16 hi, lo;
          split_bf16(h[i], hi, lo);
          h_hi[nb][s4][u] = hi;
          if constexpr (PREC == PREC_BF16X3) h_lo[nb][s4][u] = lo;
        }
      }
    }
    SSTAMP(4)
    __syncthreads();
    SSTAMP(5)
    if (t == T / 2) STACK_TL(0, 2);
  }
  SSTAMP_FLUSH(0, 0, wave == 0)
  stage(T - 1);
  __syncthreads();  // F1
  __syncthreads();  // F2 (final; the store waves have written step T-1)
  STACK_TL(0, 3);
}

// ---------------------------------------------------------------------------------------------
// forward, decoupled roles (round 6): no per-step workgroup barrier
// ---------------------------------------------------------------------------------------------
// The barrier form above makes every step as long as the slowest of its three roles: the recurrent waves' own work
// was ~1,700 of the ~2,450 cycles of a step, the rest waiting at s_barrier for input / store waves that lose the
// SIMD's issue arbitration to them (profiles/r4_lstm_f16x2_ab.txt).  Here the roles hand LDS ring slots to each other
// through per-wave monotonic step counters (the ring-gemm FULL / FREE words of MI355X_MICROARCH.md): a wave waits
// only for the slots it reads, so input and store waves run ahead / behind within their rings and the recurrent
// waves wait for each other alone (their h slices: one counter word per wave).  Every dependency is 1:1 by wave
// index w (recurrent wave w reads the gate pre-activations of units [16w, 16w + 16), written by input wave w, and
// stages its step for store wave w), except the recurrent waves' h exchange and the input waves' x image.
//
// Layer hand-off: the store waves publish the next layer's input (dropout(h), or h) as data-tagged 8-byte granules
// {value, epoch-stamped step} the moment a step is staged (no progress word, no drain); the consumer's input waves
// load and check the tags themselves (MI355X_MICROARCH.md handoff-1to1: the granule form, ~0.8-1.0 us idle, about
// half the flag form's latency).  The barrier form published a step ~5 steps after computing it and its consumer
// pre-loaded 4 steps ahead: ~10 steps (~13 us) of fill per layer boundary in each direction.
constexpr int DG = 3;   // gate pre-activation ring (input wave w -> recurrent wave w)
constexpr int HSL = 3;  // h image slots: h_t in slot (t + 1) % 3 (a wave writing h_t knows every wave read h_{t-2})
constexpr int XS = 3;   // last layer (>= 1): store wave w writes quarter w of x_{t+XS} before it stages step t
constexpr int XA = 2;   // middle layers: input wave w writes quarter w of x_{t+XA} after computing gx_t
constexpr int DX = XS + 2;  // x image slots (layers >= 1: the four quarters of x_t)
constexpr int DS = 3;   // stage slots: step t's fp32 h and BPTT stash in slot t % DS (recurrent wave w -> store wave w)
enum { SY_H = 0, SY_GX = 1, SY_STG = 2, SY_FREE = 3, SY_XQ = 4, SY_ROWS = 5 };

template <int H, int PREC>
struct FwdSmemD {
  static constexpr int ROWB = H + 8, ROWF = H + 4;
  using E = typename OpT<PREC>::E;
  float4 gxs[DG][S][H];
  E h_hi[HSL][S][PREC == PREC_F32 ? 8 : ROWB];
  __bf16 h_lo[HSL][S][PREC == PREC_BF16X3 ? ROWB : 8];
  float h_f[HSL][S][PREC == PREC_F32 ? ROWF : 4];
  E x_hi[DX][S][PREC == PREC_F32 ? 8 : ROWB];
  __bf16 x_lo[DX][S][PREC == PREC_BF16X3 ? ROWB : 8];
  float x_f[DX][S][PREC == PREC_F32 ? ROWF : 4];
  float hout[DS][S][ROWF];
  float4 st[DS][H / 16][STASH][64];
  unsigned sy[SY_ROWS][H / 16];  // per-wave step counters: [row][wave] = steps done (monotonic within a launch)
};

__device__ __forceinline__ unsigned sy_read(const unsigned* p) {
  return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wait until the NWD counters at p all reach `need` (wave-uniform; need <= 0 returns at once).  Bounded like the
// global waits: a give-up counts in the timeout word (the host raises) so the grid always drains.
template <int NWD>
__device__ __forceinline__ void sy_wait(const unsigned* p, int need, unsigned* tmo, unsigned limit) {
  if (need <= 0) return;
  for (unsigned spins = 0;; ++spins) {
    unsigned m = sy_read(p);
#pragma unroll
    for (int k = 1; k < NWD; ++k) {
      const unsigned v = sy_read(p + k);
      m = v < m ? v : m;
    }
    if ((int)__builtin_amdgcn_readfirstlane(m) >= need) break;
    if (spins >= limit) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(0);
  }
  asm volatile("" ::: "memory");  // the guarded reads are issued after the counter reads (in-order LDS)
}
// publish this wave's counter.  The LDS executes one wave's operations in issue order, so a reader that sees the
// word sees every slot write (or has every slot read) the wave issued before it: the compiler barrier keeps that
// issue order; no s_waitcnt is needed (a release fence waited lgkmcnt(0): ~150 cycles per post on the recurrent
// waves' critical path, r6 stamps)
__device__ __forceinline__ void sy_post(unsigned* p, unsigned v) {
  asm volatile("" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  asm volatile("" ::: "memory");
}

// one 8-byte granule {value bits, tag}: agent-scope relaxed load (global_load_dwordx2 sc1: L1 bypass, untorn)
__device__ __forceinline__ unsigned long long gran_load(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// two granules {v0, tag}, {v1, tag} as one 16-byte store: write-through (sc1) for a consumer on another XCD, plain
// (stays in this XCD's L2, where the consumer's sc1 loads find it) for a same-XCD consumer
__device__ __forceinline__ void gran_store2(unsigned long long* p, float v0, float v1, unsigned tag, bool local) {
  const f32x4 g{v0, __builtin_bit_cast(float, tag), v1, __builtin_bit_cast(float, tag)};
  if (local) store_plain_x4(reinterpret_cast<float*>(p), g);
  else store_sc1_x4(reinterpret_cast<float*>(p), g);
}

template <int H, int PREC, int FIN0, bool FIRST>
__device__ __forceinline__ void stack_fwd_dec(const StackFwdArgs& a, const int layer, const int tile,
                                              FwdSmemD<H, PREC>& sm, const unsigned base) {
  constexpr int NW = H / 16;
  constexpr int KB = H / 32;
  constexpr int KF = H / 4;
  constexpr int ROWB = H + 8;
  constexpr int ROWF = H + 4;
  using E = typename OpT<PREC>::E;
  using V8 = typename OpT<PREC>::V8;
  const bool last = layer == a.L - 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int role = wave / NW;  // 0 recurrent, 1 input, 2 store
  const int w = wave - role * NW;
  const int q = lane >> 4, j = lane & 15;
  const int u = 16 * w + j;
  const int n0 = tile * S;
  const int N = a.N, Np = a.Np, T = a.T;
  unsigned* const tmo = a.timeout;
  const unsigned lim = a.spin_limit;
  auto& sy = sm.sy;

  // counters and h_{-1} (image slot 0) start at zero
  for (int idx = threadIdx.x; idx < SY_ROWS * NW; idx += NW * 192) (&sy[0][0])[idx] = 0u;
  if constexpr (PREC == PREC_F32) {
    for (int idx = threadIdx.x; idx < S * ROWF; idx += NW * 192) (&sm.h_f[0][0][0])[idx] = 0.f;
  } else {
    for (int idx = threadIdx.x; idx < S * ROWB; idx += NW * 192) (&sm.h_hi[0][0][0])[idx] = (E)0.f;
    if constexpr (PREC == PREC_BF16X3)
      for (int idx = threadIdx.x; idx < S * ROWB; idx += NW * 192) (&sm.h_lo[0][0][0])[idx] = (__bf16)0.f;
  }
  __syncthreads();  // P0 (the only barrier before the final one)
  // Layers >= 1: quarter w of x_t (row ls of the tile, units lu .. lu + 3: four granules of the producer layer) goes
  // into the LDS image every input wave reads its MFMA A operand from.  Written by store wave w XS steps ahead in the
  // LAST layer (its store waves idle ~2,000 of ~2,750 cycles a step; layer 1 of L=2: forward 77.0 -> 72.7 us), by
  // input wave w XA steps ahead in a middle layer, whose store waves also produce the next layer's input (a blocking
  // upstream poll there delays every layer below: L=8 115 -> 129 us), profiles/r6_lstm_decoupled.txt.  (Each wave reading all of x_t
  // from the granules instead -- 16 scattered 8-byte loads per lane -- took ~3,000 cycles a step and crowded
  // the memory pipe: L=2 forward 79 -> 140 us, profiles/r6_lstm_decoupled.txt.)
  const int ls = lane >> 2, lu = 16 * w + 4 * (lane & 3);
  const unsigned long long* gin = FIRST ? nullptr : a.gran[layer];
  unsigned long long gq[4];
  auto issue = [&](int t) {
    const unsigned long long* p = gin + ((size_t)t * Np + n0 + ls) * H + lu;
#pragma unroll
    for (int e = 0; e < 4; ++e) gq[e] = gran_load(p + e);
  };
  auto tags_ok = [&](int t) -> bool {  // wave-uniform: the in-flight granules of step t have all arrived
    const unsigned tag = base + (unsigned)(t + 1);
    bool ok = true;
#pragma unroll
    for (int e = 0; e < 4; ++e) ok &= (unsigned)(gq[e] >> 32) == tag;
    return __builtin_amdgcn_ballot_w64(!ok) == 0;
  };
  // x_t's quarter: every lane's four tags must carry step t of this launch; reload until they do (bounded)
  auto ready = [&](int t) -> float4 {
    const unsigned tag = base + (unsigned)(t + 1);
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int e = 0; e < 4; ++e) ok &= (unsigned)(gq[e] >> 32) == tag;
      if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
      if (spins >= lim) {
        if (lane == 0) __hip_atomic_fetch_add(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      issue(t);
    }
    return make_float4(__builtin_bit_cast(float, (unsigned)gq[0]), __builtin_bit_cast(float, (unsigned)gq[1]),
                       __builtin_bit_cast(float, (unsigned)gq[2]), __builtin_bit_cast(float, (unsigned)gq[3]));
  };
  auto write_x = [&](int t, const float4& xq) {
    // image slot t % DX last held x_{t-DX}: every input wave has computed gx_{t-DX} from it
    sy_wait<NW>(&sy[SY_GX][0], t - DX + 1, tmo, lim);
    const int slot = t % DX;
    if constexpr (PREC == PREC_F32) {
      *reinterpret_cast<float4*>(&sm.x_f[slot][ls][lu]) = xq;
    } else {
      const float xv[4] = {xq.x, xq.y, xq.z, xq.w};
      if constexpr (PREC == PREC_F16X2) {
        typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
        f16x4_t v4;
#pragma unroll
        for (int e = 0; e < 4; ++e) v4[e] = (_Float16)xv[e];
        *reinterpret_cast<f16x4_t*>(&sm.x_hi[slot][ls][lu]) = v4;
      } else {
        bf16x4 hi4, lo4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          __bf16 hi, lo;
          split_bf16(xv[e], hi, lo);
          hi4[e] = hi;
          lo4[e] = lo;
        }
        *reinterpret_cast<bf16x4*>(&sm.x_hi[slot][ls][lu]) = hi4;
        if constexpr (PREC == PREC_BF16X3) *reinterpret_cast<bf16x4*>(&sm.x_lo[slot][ls][lu]) = lo4;
      }
    }
    sy_post(&sy[SY_XQ][w], t + 1);
  };

  if (role == 2) {
    // =========================== store waves ===========================
    float* hseq = a.hseq[layer];
    float4* stash = reinterpret_cast<float4*>(a.stash[layer]);
    float* xout = last ? nullptr : a.xdrop[layer + 1];
    uint32_t* mout = xout ? a.mask[layer + 1] : nullptr;
    unsigned long long* gout = last ? nullptr : a.gran[layer + 1];
    const uint32_t pseed = mout ? mta_pair_seed(a.seeds[layer + 1]) : 0;
    const float keep_scale = 1.0f / (1.0f - a.drop_p);
    const int ts = lane >> 2, tc = 4 * (lane & 3), unit4 = 16 * w + tc;
    const unsigned E = base >> a.eshift;
    if (w == 0 && lane == 0) publish_xcc(a.xcc + layer * a.tr8 + tile, E);
    const bool local = a.xcd_local && !last && partner_local(a.xcc + (layer + 1) * a.tr8 + tile, E, 1u << 14);
    // (Writing x_{t+1} blocking and x_{t+2..t+XS} only when already arrived measured slower at every depth: L=2
    // 72.7 -> 83.6 us, r6j)
    const bool sx = !FIRST && last;  // this role writes the x image (last layer)
    if (sx) {
      for (int t = 0; t < XS && t < T; ++t) {
        issue(t);
        write_x(t, ready(t));
      }
      if (XS < T) issue(XS);
    }
    SSTAMP_DECL
    for (int t = 0; t < T; ++t) {
      SSTAMP(0)
      if (sx && t + XS < T) {
        const float4 xq = ready(t + XS);
        if (t + XS + 1 < T) issue(t + XS + 1);
        write_x(t + XS, xq);
      }
      sy_wait<1>(&sy[SY_STG][w], t + 1, tmo, lim);
      SSTAMP(1)
      const int slot = t % DS;
      const float4 hv = *reinterpret_cast<const float4*>(&sm.hout[slot][ts][unit4]);
      f32x4 sv[STASH];  // (an array of HIP's float4 struct stayed in scratch memory)
      if (stash) {
#pragma unroll
        for (int k = 0; k < STASH; ++k) sv[k] = *reinterpret_cast<const f32x4*>(&sm.st[slot][w][k][lane]);
      }
      sy_post(&sy[SY_FREE][w], t + 1);  // (its fence completes the reads above)
      SSTAMP(2)
      const size_t o = ((size_t)t * Np + n0 + ts) * H + unit4;
      if (gout) {
        // the hand-off first: dropout(h) (keep bytes: pair hash, common.h) or h as tagged granules
        float4 xv = hv;
        if (xout) {
          const uint32_t kw = stack_keep_word(pseed, (uint32_t)(t * Np + n0 + ts), unit4, a.drop_p);
          xv = make_float4(hv.x * ((kw & 0xFFu) ? keep_scale : 0.f), hv.y * ((kw & 0xFF00u) ? keep_scale : 0.f),
                           hv.z * ((kw & 0xFF0000u) ? keep_scale : 0.f), hv.w * ((kw & 0xFF000000u) ? keep_scale : 0.f));
          const unsigned tag = base + (unsigned)(t + 1);
          gran_store2(gout + o, xv.x, xv.y, tag, local);
          gran_store2(gout + o + 2, xv.z, xv.w, tag, local);
          store_plain_x4(xout + o, f32x4{xv.x, xv.y, xv.z, xv.w});  // the backward's W_ih gradient input
          mout[stack_keep_index(t, tile, a.ntiles, ts, H, unit4)] = kw;
        } else {
          const unsigned tag = base + (unsigned)(t + 1);
          gran_store2(gout + o, xv.x, xv.y, tag, local);
          gran_store2(gout + o + 2, xv.z, xv.w, tag, local);
        }
      }
      store_plain_x4(hseq + o, f32x4{hv.x, hv.y, hv.z, hv.w});
      if (stash) {
#pragma unroll
        for (int k = 0; k < STASH; ++k)
          *reinterpret_cast<f32x4*>(&stash[stash_index(t, tile, a.ntiles, w, NW, lane) + 64 * k]) = sv[k];
      }
      SSTAMP(3)
    }
    SSTAMP_FLUSH(0, 1, w == 0)
    mta_wait_vmem();
    __syncthreads();  // F
    return;
  }

  float bias[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bias[g] = a.b_ih[layer][g * H + u] + a.b_hh[layer][g * H + u];

  if (role == 1) {
    // =========================== input waves ===========================
    const float* w_ih = a.w_ih[layer];
    if constexpr (FIRST) {
      float wi[4][FIN0];
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int f = 0; f < FIN0; ++f) wi[g][f] = w_ih[(g * H + u) * FIN0 + f];
      float nmask[4];
      const float* xbase[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + 4 * q + i;
        const int nr = n < N ? n : N - 1;
        nmask[i] = n < N ? 1.f : 0.f;
        if (a.gather) {
          const int K = N / a.g.B, b = nr / K, s = nr - b * K;
          const int wd = a.g.perm[a.g.cursor[0] * a.g.B + b];
          xbase[i] = a.g.src[0] + (size_t)wd * a.g.row[0] + (size_t)s * T * FIN0;
        } else {
          xbase[i] = a.x + (size_t)nr * T * FIN0;
        }
      }
      struct XBuf {
        float x0[4][FIN0];
      };
      XBuf xbA, xbB;
      auto load_input = [&](int t, XBuf& xb) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int f = 0; f < FIN0; ++f) xb.x0[i][f] = xbase[i][(size_t)t * FIN0 + f];
      };
      // interval t: gx_t from the set loaded two intervals ago, then refill it with x_{t+2}
      SSTAMP_DECL
      auto body = [&](int t, XBuf& xb) {
        SSTAMP(0)
        sy_wait<1>(&sy[SY_H][w], t - DG + 1, tmo, lim);  // slot t % DG: recurrent wave w read gx_{t-DG}
        SSTAMP(1)
        const int slot = t % DG;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float acc[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float sacc = bias[g];
#pragma unroll
            for (int f = 0; f < FIN0; ++f) sacc = fmaf(xb.x0[i][f] * nmask[i], wi[g][f], sacc);
            acc[g] = sacc;
          }
          sm.gxs[slot][4 * q + i][u] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
        sy_post(&sy[SY_GX][w], t + 1);
        SSTAMP(2)
        if (t + 2 < T) load_input(t + 2, xb);
        SSTAMP(3)
      };
      load_input(0, xbA);
      if (T > 1) load_input(1, xbB);
      for (int t = 0; t < T; t += 2) {
        body(t, xbA);
        if (t + 1 < T) body(t + 1, xbB);
      }
      SSTAMP_FLUSH(0, 2, w == 0)
    } else {
      constexpr int XKB = KB, XKF = KF;
      V8 Xhi[4][PREC == PREC_F32 ? 1 : XKB], Xlo[4][kWeightLo<PREC> ? XKB : 1];
      float Xf[4][PREC == PREC_F32 ? XKF : 1];
      if constexpr (PREC == PREC_F32) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int kk = 0; kk < KF; ++kk) Xf[g][kk] = w_ih[(size_t)(g * H + u) * H + KF * q + kk];
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              E hi, lo;
              split_bf16(w_ih[(size_t)(g * H + u) * H + 32 * kb + 8 * q + e], hi, lo);
              Xhi[g][kb][e] = hi;
              if constexpr (kWeightLo<PREC>) Xlo[g][kb][e] = lo;
            }
      }
      auto compute_gx_img = [&](int t) {
        const int xs = t % DX, slot = t % DG;
        f32x4 acc[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = f32x4{bias[g], bias[g], bias[g], bias[g]};
        if constexpr (PREC == PREC_F32) {
          const float* xr = &sm.x_f[xs][j][KF * q];
#pragma unroll
          for (int kk = 0; kk < KF; ++kk) {
            const float av = xr[kk];
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[g] = mfma16x16x4f32(av, Xf[g][kk], acc[g]);
          }
        } else {
          V8 ahi[KB];
          bf16x8 alo[PREC == PREC_BF16X3 ? KB : 1];
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
            ahi[kb] = *reinterpret_cast<const V8*>(&sm.x_hi[xs][j][32 * kb + 8 * q]);
            if constexpr (PREC == PREC_BF16X3) alo[kb] = *reinterpret_cast<const bf16x8*>(&sm.x_lo[xs][j][32 * kb + 8 * q]);
          }
#pragma unroll
          for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              if constexpr (PREC == PREC_BF16X3) {
                acc[g] = mfma16x16x32(alo[kb], Xhi[g][kb], acc[g]);
                acc[g] = mfma16x16x32(ahi[kb], Xlo[g][kb], acc[g]);
              }
              if constexpr (PREC == PREC_F16X2) acc[g] = mfma16x16x32(ahi[kb], Xlo[g][kb], acc[g]);
              acc[g] = mfma16x16x32(ahi[kb], Xhi[g][kb], acc[g]);
            }
        }
        sy_wait<1>(&sy[SY_H][w], t - DG + 1, tmo, lim);  // gx slot: recurrent wave w read gx_{t-DG}
#pragma unroll
        for (int i = 0; i < 4; ++i)
          sm.gxs[slot][4 * q + i][u] = make_float4(acc[0][i], acc[1][i], acc[2][i], acc[3][i]);
        sy_post(&sy[SY_GX][w], t + 1);
      };
      // iteration t: gx_t from x_t's image; a middle layer's input wave then writes its quarter of x_{t+XA} (granules
      // issued an iteration ago), the last layer's store waves write the image XS steps ahead
      const bool ix = !last;
      if (ix) {
        for (int t = 0; t < XA && t < T; ++t) {
          issue(t);
          write_x(t, ready(t));
        }
        if (XA < T) issue(XA);
      }
      SSTAMP_DECL
      for (int t = 0; t < T; ++t) {
        SSTAMP(0)
        sy_wait<NW>(&sy[SY_XQ][0], t + 1, tmo, lim);  // x_t's image complete (all four quarters)
        SSTAMP(1)
        compute_gx_img(t);
        SSTAMP(2)
        if (ix && t + XA < T) {
          const float4 xq = ready(t + XA);
          SSTAMP(3)
          if (t + XA + 1 < T) issue(t + XA + 1);
          write_x(t + XA, xq);
          SSTAMP(4)
        }
      }
      SSTAMP_FLUSH(0, 2, w == 0)
    }
    __syncthreads();  // F
    return;
  }

  // =========================== recurrent waves ===========================
  if (__builtin_amdgcn_readfirstlane(wave) < NW) __builtin_amdgcn_s_setprio(STACK_PRIO);
  STACK_TL(0, 0);
  const float* w_hh = a.w_hh[layer];
  const bool stash = a.stash[layer] != nullptr;
  V8 Bhi[4][PREC == PREC_F32 ? 1 : KB], Blo[4][kWeightLo<PREC> ? KB : 1];
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
          E hi, lo;
          split_bf16(w_hh[(size_t)(g * H + u) * H + 32 * kb + 8 * q + e], hi, lo);
          Bhi[g][kb][e] = hi;
          if constexpr (kWeightLo<PREC>) Blo[g][kb][e] = lo;
        }
  }
  float c[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 pgi, pgf, pgg, pgo, pcc;
  float h[4];
  // step t's fp32 h and BPTT stash -> stage slot t % DS (store wave w read step t - DS out of it first; free_seen:
  // its counter as read with the step's batch)
  unsigned free_seen = 0;
  auto stage = [&](int t) {
    if ((int)__builtin_amdgcn_readfirstlane(free_seen) < t - DS + 1) sy_wait<1>(&sy[SY_FREE][w], t - DS + 1, tmo, lim);
    const int slot = t % DS;
#pragma unroll
    for (int i = 0; i < 4; ++i) sm.hout[slot][4 * q + i][u] = h[i];
    if (stash) {
      sm.st[slot][w][0][lane] = make_float4(pgi[0], pgi[1], pgi[2], pgi[3]);
      sm.st[slot][w][1][lane] = make_float4(pgf[0], pgf[1], pgf[2], pgf[3]);
      sm.st[slot][w][2][lane] = make_float4(pgg[0], pgg[1], pgg[2], pgg[3]);
      sm.st[slot][w][3][lane] = make_float4(pgo[0], pgo[1], pgo[2], pgo[3]);
      sm.st[slot][w][4][lane] = make_float4(pcc[0], pcc[1], pcc[2], pcc[3]);
    }
  };
  SSTAMP_DECL
  // A step reads its counters and the slots they guard in ONE batch (counters first: the LDS serves a wave's reads in
  // order, so a slot read issued after a counter that shows it ready returns its final content) and waits once; only
  // when a counter is behind does it poll and re-read (rare: the input waves run DG steps ahead, and the h counters
  // of the four recurrent waves are usually all posted by the time the batch is served).  Polling first and reading
  // after cost two LDS round trips per dependency (~600 of ~2,460 cycles a step, r6 stamps).
  f32x4 acc[4];
  V8 ahi[PREC == PREC_F32 ? 1 : KB];
  bf16x8 alo[PREC == PREC_BF16X3 ? KB : 1];
  auto read_gx = [&](int t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 v = sm.gxs[t % DG][4 * q + i][u];
      acc[0][i] = v.x;
      acc[1][i] = v.y;
      acc[2][i] = v.z;
      acc[3][i] = v.w;
    }
  };
  auto read_a = [&](int hs) {
    if constexpr (PREC != PREC_F32) {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        ahi[kb] = *reinterpret_cast<const V8*>(&sm.h_hi[hs][j][32 * kb + 8 * q]);
        if constexpr (PREC == PREC_BF16X3) alo[kb] = *reinterpret_cast<const bf16x8*>(&sm.h_lo[hs][j][32 * kb + 8 * q]);
      }
    }
  };
  STACK_TL(0, 1);
  for (int t = 0; t < T; ++t) {
    SSTAMP(0)
    const int hs = t % HSL, hn = (t + 1) % HSL;
    const unsigned cg = sy_read(&sy[SY_GX][w]);  // gx_t of this wave's units
    unsigned hmin = 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < NW; ++k) {  // every recurrent wave's slice of h_{t-1}
      const unsigned v = sy_read(&sy[SY_H][k]);
      hmin = v < hmin ? v : hmin;
    }
    free_seen = sy_read(&sy[SY_FREE][w]);  // the stage slot of step t-1 (checked by stage())
    asm volatile("" ::: "memory");
    read_gx(t);
    read_a(hs);
    SSTAMP(1)
    if ((int)__builtin_amdgcn_readfirstlane(cg) < t + 1 || (int)__builtin_amdgcn_readfirstlane(hmin) < t) {
      sy_wait<1>(&sy[SY_GX][w], t + 1, tmo, lim);
      sy_wait<NW>(&sy[SY_H][0], t, tmo, lim);
      read_gx(t);
      read_a(hs);
    }
    SSTAMP(2)
    if constexpr (PREC == PREC_F32) {
      if (t > 0) {
        stage(t - 1);
        sy_post(&sy[SY_STG][w], (unsigned)t);  // (the store waves start on it a whole MFMA chain earlier)
      }
      const float* hrow = &sm.h_f[hs][j][q * KF];
#pragma unroll
      for (int kk = 0; kk < KF; ++kk) {
        const float av = hrow[kk];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = mfma16x16x4f32(av, Bf[g][kk], acc[g]);
      }
    } else {
      if (t > 0) {
        stage(t - 1);
        sy_post(&sy[SY_STG][w], (unsigned)t);  // (the store waves start on it a whole MFMA chain earlier)
      }
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
        for (int sg = 0; sg < kPasses<PREC>; ++sg) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            if constexpr (PREC == PREC_BF16X3) {
              if (sg == 0) acc[g] = mfma16x16x32(alo[kb], Bhi[g][kb], acc[g]);
              else if (sg == 1) acc[g] = mfma16x16x32(ahi[kb], Blo[g][kb], acc[g]);
              else acc[g] = mfma16x16x32(ahi[kb], Bhi[g][kb], acc[g]);
            } else if constexpr (PREC == PREC_F16X2) {
              if (sg == 0) acc[g] = mfma16x16x32(ahi[kb], Blo[g][kb], acc[g]);
              else acc[g] = mfma16x16x32(ahi[kb], Bhi[g][kb], acc[g]);
            } else {
              acc[g] = mfma16x16x32(ahi[kb], Bhi[g][kb], acc[g]);
            }
          }
        }
      }
    }
    // (step t-1's stage slot is posted right after it is written, above: posting it behind the MFMA chain cost
    // 0.3 / 1.0 / 2.0 us at L = 2 / 4 / 8, profiles/r6_lstm_dec/r7d_probe.txt)
    __builtin_amdgcn_sched_barrier(0);
    SSTAMP(3)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pgi[i] = mta_sigmoid(acc[0][i]);
      pgf[i] = mta_sigmoid(acc[1][i]);
      pgg[i] = mta_tanh(acc[2][i]);
      pgo[i] = mta_sigmoid(acc[3][i]);
      c[i] = fmaf(pgf[i], c[i], pgi[i] * pgg[i]);
      pcc[i] = c[i];
      h[i] = pgo[i] * mta_tanh(c[i]);
    }
    SSTAMP(4)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s4 = 4 * q + i;
      if constexpr (PREC == PREC_F32) {
        sm.h_f[hn][s4][(u & 3) * KF + (u >> 2)] = h[i];
      } else if constexpr (PREC == PREC_F16X2) {
        sm.h_hi[hn][s4][u] = (_Float16)h[i];
      } else {
        __bf16 hi, lo;
        split_bf16(h[i], hi, lo);
        sm.h_hi[hn][s4][u] = hi;
        if constexpr (PREC == PREC_BF16X3) sm.h_lo[hn][s4][u] = lo;
      }
    }
    sy_post(&sy[SY_H][w], (unsigned)(t + 1));
    SSTAMP(5)
    if (t == T / 2) STACK_TL(0, 2);
  }
  SSTAMP_FLUSH(0, 0, wave == 0)
  stage(T - 1);
  sy_post(&sy[SY_STG][w], (unsigned)T);
  STACK_TL(0, 3);
  __syncthreads();  // F
}

// batch rows -> static buffers, spread over workgroups [0, P) (the gather of csrc/lstm_aux.hip, in this launch);
// four independent 16-byte loads in flight per thread before their stores
__device__ __forceinline__ void batch_copy(const MtaBatchGather& g, int p, int P) {
  // 32-bit indices (a batch is B x row floats, far below 2^31): the 64-bit division's two-path expansion branched
  // around the loads and kept v[] in scratch memory
  const int cur = g.cursor[0];
  const int stride = P * (int)blockDim.x, first = p * (int)blockDim.x + (int)threadIdx.x;
  for (int k = 0; k < g.nt; ++k) {
    const int row = (int)g.row[k], total = g.B * row;
    if ((row & 3) == 0 && ((((uintptr_t)g.src[k]) | ((uintptr_t)g.dst[k])) & 15) == 0) {
      const int row4 = row / 4, n4 = total / 4;
      const f32x4* s4 = reinterpret_cast<const f32x4*>(g.src[k]);
      f32x4* d4 = reinterpret_cast<f32x4*>(g.dst[k]);
      for (int e0 = first; e0 < n4; e0 += 4 * stride) {
        f32x4 v[4];  // (HIP's float4 struct kept this array in scratch memory)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = e0 + r * stride < n4 ? e0 + r * stride : n4 - 1;  // clamped, unconditional
          const int b = e / row4;
          v[r] = s4[(size_t)g.perm[cur * g.B + b] * row4 + (e - b * row4)];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (e0 + r * stride < n4) d4[e0 + r * stride] = v[r];
      }
    } else {
      for (int e = first; e < total; e += stride) {
        const int b = e / row;
        g.dst[k][e] = g.src[k][(size_t)g.perm[cur * g.B + b] * row + (e - b * row)];
      }
    }
  }
}

template <int H, int PREC, int FIN0, bool DEC>
__global__ __launch_bounds__((H / 16) * 192) void lstm_stack_fwd_kernel(StackFwdArgs a) {
  // layer l's workgroups follow layer l-1's in block-id order (its producers are already resident)
  if ((int)blockIdx.x >= a.main_blocks) {
    // batch-copy workgroup (gather mode): no hand-offs, only the copy and the launch arrival
    const unsigned cbase = read_epoch_base(a.ctl, CTL_FWD_EPOCH, a.eshift);
    batch_copy(a.g, blockIdx.x - a.main_blocks, a.copy_blocks);
    if (finish_launch(a.ctl, CTL_FWD_EPOCH, CTL_FWD_DONE, cbase, a.eshift)) a.g.cursor[0] += 1;
    return;
  }
  const int layer = blockIdx.x / a.tr8, tile = blockIdx.x % a.tr8;
  const unsigned base = read_epoch_base(a.ctl, CTL_FWD_EPOCH, a.eshift);
  if constexpr (DEC) {
    __shared__ __attribute__((aligned(16))) FwdSmemD<H, PREC> sm;  // one image shared by both role bodies
    if (tile < a.ntiles) {
      if (layer == 0) stack_fwd_dec<H, PREC, FIN0, true>(a, layer, tile, sm, base);
      else stack_fwd_dec<H, PREC, FIN0, false>(a, layer, tile, sm, base);
    }
  } else {
    __shared__ __attribute__((aligned(16))) FwdSmem<H, PREC> sm;  // one image shared by both role bodies
    if (tile < a.ntiles) {
      if (layer == 0) stack_fwd_body<H, PREC, FIN0, true>(a, layer, tile, sm, base);
      else stack_fwd_body<H, PREC, FIN0, false>(a, layer, tile, sm, base);
    }
  }
  // every workgroup read the cursor before arriving: the last one advances it
  if (finish_launch(a.ctl, CTL_FWD_EPOCH, CTL_FWD_DONE, base, a.eshift) && a.gather) a.g.cursor[0] += 1;
}

// ---------------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------------
template <int H>
__device__ __forceinline__ int rperm_to_r(int rp) {
  const int e = rp & 7, p = rp >> 3;
  const int uu = 2 * p + (e >> 2), g = e & 3;
  return g * H + uu;
}

struct StackBwdArgs {
  const float* stash[MAXL];
  const float* w_hh[MAXL];
  const float* w_ih[MAXL];
  const float* dh_last;   // (N, H): gradient wrt h_{T-1} of the top layer
  float* dG[MAXL];        // (T, Np, 4H) per layer, unit-major columns
  float* dX[MAXL];        // dX[l] (l < L-1): gradient wrt layer l's output sequence, written by layer l+1
  const uint32_t* mask[MAXL];  // mask[l] (l >= 1, dropout): keep-byte words of layer l's input dropout (fwd)
  uint64_t* seeds;        // [MAXL]: dropout seed of layer l's input (advanced by the launch's last workgroup)
  float drop_p;
  int dropout;
  unsigned* flags;        // [MAXL][tr8]: reverse steps of dX[l-1] published by layer l
  unsigned* dg_flags;     // [MAXL][tr8]: reverse steps of dG[l] drained (write-through) by layer l
  unsigned* timeout;
  unsigned* ctl;
  unsigned spin_limit;
  int N, Np, T, L, ntiles, tr8, eshift;
  // fused weight gradients: wg_per_layer workgroups per layer follow the L x tr8 recurrence workgroups
  mta_wgrad::WgArgs wg[MAXL];
  int wg_nq, wg_per_layer;
};

template <int H, int PREC>
struct BwdSmem {
  static constexpr int ROWB = 4 * H + 8, ROWF = 4 * H + 4;
  __bf16 g_hi[2][S][PREC == PREC_F32 ? 8 : ROWB];
  __bf16 g_lo[2][S][PREC == PREC_BF16X3 ? ROWB : 8];
  float g_f[2][S][PREC == PREC_F32 ? ROWF : 4];
  float dhs[2][S][H];  // dH_t of the layer above, staged by the gradient waves
  float tr[H / 16][S][TRS];  // per-gradient-wave transpose scratch of the dx store
};

// Backward workgroup = 2 x (H/16) waves.  Waves [0, H/16) run BPTT exactly like lstm.hip (dG_t from the
// stash, dh_{t-1} = dG_t W_hh through the LDS dG image, one barrier per step); waves [H/16, 2 H/16) are
// GRADIENT waves: they stage dH_t of the layer above into LDS two steps ahead (progress polls and hand-off
// latency off the recurrent path) and compute dx_t = dG_t W_ih from the same LDS image one step behind,
// apply this layer's input-dropout mask and hand dH^{(l-1)} to the layer below.
// Intervals: I(t) = between barriers A(t+1) and A(t); the recurrent waves read dhs[t&1] and write the
// dG image (t&1) in I(t); the gradient waves write dhs[(t-1)&1] and read image ((t+1)&1) in I(t).
// DPF: how many intervals before its staging a gradient wave loads dH of the layer above -- 1 (L <= 2: the least
// fill per layer) or 2 (deeper stacks: the hand-off round trip off every lower layer's interval; L=4 144 -> 132 us,
// L=8 203 -> 186 us, L=2 92 -> 95 us, profiles/r6_lstm_dec/r6u_probe.txt)
template <int H, int PREC, bool TOP, bool BOTTOM, int DPF>
__device__ __forceinline__ void stack_bwd_body(const StackBwdArgs& a, const int layer, const int tile,
                                               BwdSmem<H, PREC>& sm, const unsigned base) {
  constexpr int G4 = 4 * H;
  constexpr int NW = H / 16;
  constexpr int KB = G4 / 32;
  constexpr int KF = G4 / 4;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool grad_wave = wave >= NW;
  const int w = grad_wave ? wave - NW : wave;
  const int q = lane >> 4, j = lane & 15;
  const int u = 16 * w + j;
  const int n0 = tile * S;
  const int N = a.N, Np = a.Np, T = a.T;
  auto& g_hi = sm.g_hi;
  auto& g_lo = sm.g_lo;
  auto& g_f = sm.g_f;
  auto& dhs = sm.dhs;

  if (grad_wave) {
    // =========================== gradient waves ===========================
    const float* dH = TOP ? nullptr : a.dX[layer];
    float* dXout = BOTTOM ? nullptr : a.dX[layer - 1];
    const uint32_t* min = (!BOTTOM && a.dropout) ? a.mask[layer] : nullptr;
    const float keep_scale = 1.0f / (1.0f - a.drop_p);
    unsigned* my_flag = a.flags + FLAG_STRIDE * (layer * a.tr8 + tile);
    unsigned* in_flag = TOP ? my_flag : a.flags + FLAG_STRIDE * ((layer + 1) * a.tr8 + tile);
    unsigned* dg_flag = a.dg_flags + FLAG_STRIDE * (layer * a.tr8 + tile);
    const float* w_ih = a.w_ih[layer];
    float* dG = a.dG[layer];
    constexpr int XKB = BOTTOM ? 1 : KB, XKF = BOTTOM ? 1 : KF;
    bf16x8 Xhi[PREC == PREC_F32 ? 1 : XKB], Xlo[PREC == PREC_BF16X3 ? XKB : 1];
    float Xf[PREC == PREC_F32 ? XKF : 1];
    if constexpr (!BOTTOM) {
      if constexpr (PREC == PREC_F32) {
#pragma unroll
        for (int kk = 0; kk < KF; ++kk) Xf[kk] = w_ih[(size_t)(4 * kk + q) * H + u];
      } else {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            __bf16 hi, lo;
            split_bf16(w_ih[(size_t)rperm_to_r<H>(32 * kb + 8 * q + e) * H + u], hi, lo);
            Xhi[kb][e] = hi;
            if constexpr (PREC == PREC_BF16X3) Xlo[kb][e] = lo;
          }
      }
    }
    // dH_s of the layer above (4 sequences x unit u) into one of two register sets, loaded DPF intervals before it
    // is staged
    float dA[4] = {0.f, 0.f, 0.f, 0.f}, dB[4] = {0.f, 0.f, 0.f, 0.f};
    unsigned seen = base;
    auto load_dh = [&](int t, float (&d)[4]) {
      if constexpr (!TOP) {
        seen = wait_progress(in_flag, base + (unsigned)(T - t), seen, a.timeout, a.spin_limit);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          d[i] = __hip_atomic_load(const_cast<float*>(dH) + ((size_t)t * Np + n0 + 4 * q + i) * H + u,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    };
    uint32_t mreg = 0x01010101u, mnext = 0x01010101u;
    const int ts = lane >> 2, tc = 4 * (lane & 3);
    auto load_mask = [&](int t) {  // keep bytes of step t (row ts, units 16 w + tc + e), used one interval later
      if constexpr (!BOTTOM) {
        if (min) mnext = min[stack_keep_index(t, tile, a.ntiles, ts, H, 16 * w + tc)];
      }
    };
    auto stage_dh = [&](int t, const float (&d)[4]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dhs[t & 1][4 * q + i][u] = d[i];
    };
    auto dx_step = [&](int t) {  // dG_t stores and dx_t = dG_t . W_ih from image (t&1) -> masked sc1 stores
      if constexpr (!BOTTOM) {
        const int buf = t & 1;
        // four independent accumulation chains (even / odd k-blocks x hi / cross terms)
        f32x4 ax[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
        if constexpr (PREC == PREC_F32) {
          const float* arow = &g_f[buf][j][q * KF];
#pragma unroll
          for (int kk = 0; kk < KF; ++kk) ax[kk & 3] = mfma16x16x4f32(arow[kk], Xf[kk], ax[kk & 3]);
        } else {
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
            const bf16x8 ahi = *reinterpret_cast<const bf16x8*>(&g_hi[buf][j][32 * kb + 8 * q]);
            if constexpr (PREC == PREC_BF16X3) {
              const bf16x8 alo = *reinterpret_cast<const bf16x8*>(&g_lo[buf][j][32 * kb + 8 * q]);
              ax[2 + (kb & 1)] = mfma16x16x32(alo, Xhi[kb], ax[2 + (kb & 1)]);
              ax[2 + (kb & 1)] = mfma16x16x32(ahi, Xlo[kb], ax[2 + (kb & 1)]);
            }
            ax[kb & 1] = mfma16x16x32(ahi, Xhi[kb], ax[kb & 1]);
          }
        }
        // one 16-byte write-through store per lane (transpose through the wave's own LDS scratch); the input
        // dropout mask (keep words in this store layout) is applied after the transpose
        float (*tr)[TRS] = sm.tr[w];
#pragma unroll
        for (int i = 0; i < 4; ++i) tr[4 * q + i][j] = (ax[0][i] + ax[1][i]) + (ax[2][i] + ax[3][i]);
        const float4 dv = *reinterpret_cast<const float4*>(&tr[ts][tc]);
        f32x4 o{dv.x, dv.y, dv.z, dv.w};
        if (min) {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] *= ((mreg >> (8 * e)) & 0xFFu) ? keep_scale : 0.f;
        }
        store_sc1_x4(dXout + ((size_t)t * Np + n0 + ts) * H + 16 * w + tc, o);
      }
    };
    // interval I(t) (sets X, Y; DPF 2: they swap every interval -- a loop of exactly two intervals per trip keeps each
    // set in its registers): DPF 2 stages dH_{t-1} out of X (loaded in I(t+2)) and loads dH_{t-3} into it again;
    // DPF 1 (X = Y, one set) stages dH_{t-1} (loaded in I(t+1)) and loads dH_{t-2}
    if constexpr (!TOP) {
      load_dh(T - 1, dA);
      stage_dh(T - 1, dA);
      if constexpr (DPF == 2) {
        if (T > 1) load_dh(T - 2, dA);
        if (T > 2) load_dh(T - 3, dB);
      } else {
        if (T > 1) load_dh(T - 2, dA);
      }
    }
    __syncthreads();  // B0
    SSTAMP_DECL
    auto interval = [&](int t, float (&X)[4], float (&Y)[4]) {
      // ---- interval I(t) ----  issue order: [keep-byte load, dH loads, dx store].  The dx product runs last,
      // while the recurrent waves are in their VALU phase (their dh MFMAs run right after A(t+1); two MFMA streams
      // on one SIMD serialise, r2 stamp probe), and its store stays in flight across the barrier.
      SSTAMP(0)
      // every op older than the previous interval's dx store (DPF 2: its dH loads + dx store) is complete: its keep
      // word (used now), the dx stores of I(t+2) and earlier (the progress word below)
      if constexpr (TOP && BOTTOM) mta_wait_vmem();
      else if constexpr (BOTTOM) mta_wait_vmcnt<DPF == 2 ? 4 : 0>();
      else if constexpr (TOP) mta_wait_vmcnt<1>();
      else mta_wait_vmcnt<DPF == 2 ? 5 : 1>();
      mreg = mnext;
      SSTAMP(1)
      // progress: dx of steps >= t+4 (stored in I(t+3) or earlier) was drained by every gradient wave's wait at
      // the top of I(t+1) (which leaves only I(t+2)'s loads and store in flight), before barrier A(t+1).  (Publishing
      // a step earlier from per-wave LDS drain counters + atomic-max progress words was slower at every depth: L=2
      // 86.3 -> 91.0 us, L=8 192 -> 199, profiles/r6_lstm_dec/r7c_probe.txt)
      if (!BOTTOM && t + 4 <= T - 1 && wave == NW && lane == 0)
        __hip_atomic_store(my_flag, base + (unsigned)(T - t - 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // dG progress: the recurrent waves store dG_{s} in their step s-1 and pass their vmcnt(10) wait at the top of
      // step s-3 only once those stores are complete, before barrier A(s-3): at I(t) (after A(t+1)) every dG_s with
      // s >= t+4 is drained
      if (t + 4 <= T - 1 && wave == NW + 1 && lane == 0)
        __hip_atomic_store(dg_flag, base + (unsigned)(T - t - 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      load_mask(t);  // for dx_step(t) in I(t-1)
      if constexpr (!TOP) {
        if constexpr (DPF == 2) {
          if (t >= 1) stage_dh(t - 1, X);
          if (t >= 3) load_dh(t - 3, X);
        } else {
          if (t >= 1) stage_dh(t - 1, Y);
          if (t >= 2) load_dh(t - 2, X);
        }
      }
      SSTAMP(2)
      // (stacks of 3+ layers start the dx product at once: L=4 bwd 127.4 -> 123.6 us, L=8 unchanged;
      // profiles/r6_lstm_dec/r7h_probe.txt)
      if constexpr (!BOTTOM && DPF == 1) __builtin_amdgcn_s_sleep(DX_DELAY);
      if (t + 1 <= T - 1) dx_step(t + 1);
      SSTAMP(3)
      __syncthreads();  // A(t)
      SSTAMP(4)
    };
    if constexpr (DPF == 2) {
      int t = T - 1;
      for (; t >= 1; t -= 2) {
        interval(t, dA, dB);
        interval(t - 1, dB, dA);
      }
      if (t == 0) interval(0, dA, dB);
    } else {
      // one set (staged, then reloaded, in the same interval): no unrolled copy of the interval (the two-interval
      // loop cost ~2.4 us at L=2, instruction footprint; profiles/r6_lstm_dec/r6x_probe.txt)
      for (int t = T - 1; t >= 0; --t) interval(t, dA, dA);
    }
    SSTAMP_FLUSH(1, 1, w == 0)
    mta_wait_vmem();
    mreg = mnext;
    dx_step(0);
    mta_wait_vmem();
    __syncthreads();  // F
    if (!BOTTOM && wave == NW && lane == 0)
      __hip_atomic_store(my_flag, base + (unsigned)T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wave == NW + 1 && lane == 0)
      __hip_atomic_store(dg_flag, base + (unsigned)T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }

  // =========================== recurrent waves ===========================
  if (__builtin_amdgcn_readfirstlane(wave) < NW) __builtin_amdgcn_s_setprio(STACK_PRIO);
  STACK_TL(1, 0);
  const float4* stash = reinterpret_cast<const float4*>(a.stash[layer]);
  const float* w_hh = a.w_hh[layer];
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
        __bf16 hi, lo;
        split_bf16(w_hh[(size_t)rperm_to_r<H>(32 * kb + 8 * q + e) * H + u], hi, lo);
        Bhi[kb][e] = hi;
        if constexpr (PREC == PREC_BF16X3) Blo[kb][e] = lo;
      }
  }
  float dc[4] = {0.f, 0.f, 0.f, 0.f};
  float dhr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + 4 * q + i;
    if constexpr (TOP) {
      const float v = a.dh_last[(size_t)(n < N ? n : N - 1) * H + u];
      dhr[i] = n < N ? v : 0.f;
    } else {
      dhr[i] = 0.f;
    }
  }
  float pdG[4][4] = {};
  [[maybe_unused]] float* dG = a.dG[layer];
  auto store_step = [&](int t) {  // write-through dG rows from the recurrent waves
#pragma unroll
    for (int i = 0; i < 4; ++i)
      store_sc1_x4(dG + ((size_t)t * Np + n0 + 4 * q + i) * G4 + 4 * u,
                   f32x4{pdG[0][i], pdG[1][i], pdG[2][i], pdG[3][i]});
  };
  // stash of step t (i, f, g, o, c) plus c_{t-1}, prefetched ~two steps ahead into one of two register
  // sets (even / odd steps); a step issues the 6 stash loads of step t-2 (mode 0: after the 4 dG stores of step
  // t+1), so at the top of step t the loads it needs are followed by exactly 6 (mode 0: 10) newer ops
  auto load_into = [&](int t, float4 (&sb)[STASH], float4& cb) {
    const float4* src = stash + stash_index(t, tile, a.ntiles, w, NW, lane);
#pragma unroll
    for (int k = 0; k < STASH; ++k) sb[k] = src[64 * k];
    cb = stash[stash_index(t > 0 ? t - 1 : 0, tile, a.ntiles, w, NW, lane) + 64 * 4];
  };
  float4 sA[STASH], cA, sB[STASH], cB;
  load_into(T - 1, sA, cA);
  if (T > 1) load_into(T - 2, sB, cB);
  __syncthreads();  // B0 (dhs[(T-1)&1] staged)

  // one reverse step; returns false after step 0
  SSTAMP_DECL
  auto step = [&](int t, float4 (&sb)[STASH], float4& cb) {
    SSTAMP(0)
    float dho[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) dho[i] = TOP ? 0.f : dhs[t & 1][4 * q + i][u];
    SSTAMP(1)
    if (t <= T - 2) mta_wait_vmcnt<10>();
    else mta_wait_vmcnt<6>();
    SSTAMP(2)
    // unconditional (step T-1 stores its zero pdG to row T-1, which step T-2 then overwrites in order)
    store_step(t < T - 1 ? t + 1 : t);
    __builtin_amdgcn_sched_barrier(0);
    SSTAMP(3)
    const float4* st = sb;
    const float cpm = t > 0 ? 1.f : 0.f;
    const float cp4[4] = {cb.x * cpm, cb.y * cpm, cb.z * cpm, cb.w * cpm};
    const float ig4[4] = {st[0].x, st[0].y, st[0].z, st[0].w};
    const float fg4[4] = {st[1].x, st[1].y, st[1].z, st[1].w};
    const float gg4[4] = {st[2].x, st[2].y, st[2].z, st[2].w};
    const float og4[4] = {st[3].x, st[3].y, st[3].z, st[3].w};
    const float ct4[4] = {st[4].x, st[4].y, st[4].z, st[4].w};
    const int buf = t & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float ig = ig4[i], fg = fg4[i], gg = gg4[i], og = og4[i];
      const float dh = dho[i] + dhr[i];
      const float tc = mta_tanh(ct4[i]);
      const float d_o = dh * tc * og * (1.f - og);
      const float dcc = fmaf(dh * og, 1.f - tc * tc, dc[i]);
      pdG[0][i] = dcc * gg * ig * (1.f - ig);
      pdG[1][i] = dcc * cp4[i] * fg * (1.f - fg);
      pdG[2][i] = dcc * ig * (1.f - gg * gg);
      pdG[3][i] = d_o;
      dc[i] = dcc * fg;
      const int s4 = 4 * q + i;
      if constexpr (PREC == PREC_F32) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int r = g * H + u;
          g_f[buf][s4][(r & 3) * KF + (r >> 2)] = pdG[g][i];
        }
      } else {
        bf16x4 hi4, lo4;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          __bf16 hi, lo;
          split_bf16(pdG[g][i], hi, lo);
          hi4[g] = hi;
          lo4[g] = lo;
        }
        const int rp = 8 * (u >> 1) + 4 * (u & 1);
        *reinterpret_cast<bf16x4*>(&g_hi[buf][s4][rp]) = hi4;
        if constexpr (PREC == PREC_BF16X3) *reinterpret_cast<bf16x4*>(&g_lo[buf][s4][rp]) = lo4;
      }
    }
    SSTAMP(4)
    // prefetch step t-2 into this set (its values are dead now); unconditional, so the set needs no copy
    __builtin_amdgcn_sched_barrier(0);
    load_into(t >= 2 ? t - 2 : 0, sb, cb);
    SSTAMP(5)
    __syncthreads();  // A(t): dG_t image visible to the gradient waves and to this step's dh product
    SSTAMP(6)
    if (t == 0) return;
    // four independent accumulation chains (even / odd k-blocks x hi / cross terms): the dependent-MFMA
    // latency, not issue, bounded the two-chain form (r2 stamp probe: 795 cycles for 24 MFMAs)
    f32x4 ac[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if constexpr (PREC == PREC_F32) {
      const float* arow = &g_f[buf][j][q * KF];
#pragma unroll
      for (int kk = 0; kk < KF; ++kk) ac[kk & 3] = mfma16x16x4f32(arow[kk], Bf[kk], ac[kk & 3]);
    } else {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const bf16x8 ahi = *reinterpret_cast<const bf16x8*>(&g_hi[buf][j][32 * kb + 8 * q]);
        if constexpr (PREC == PREC_BF16X3) {
          const bf16x8 alo = *reinterpret_cast<const bf16x8*>(&g_lo[buf][j][32 * kb + 8 * q]);
          ac[2 + (kb & 1)] = mfma16x16x32(alo, Bhi[kb], ac[2 + (kb & 1)]);
          ac[2 + (kb & 1)] = mfma16x16x32(ahi, Blo[kb], ac[2 + (kb & 1)]);
        }
        ac[kb & 1] = mfma16x16x32(ahi, Bhi[kb], ac[kb & 1]);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) dhr[i] = (ac[0][i] + ac[1][i]) + (ac[2][i] + ac[3][i]);
    SSTAMP(7)
  };
  // steps T-1, T-3, ... use set A; T-2, T-4, ... set B: a loop of exactly two steps per trip (no
  // conditional step inside, so the sets keep their registers across the back-edge), odd T peels step 0
  STACK_TL(1, 1);
  int t = T - 1;
  for (; t >= 1; t -= 2) {
    step(t, sA, cA);
    if (t == T / 2 || t - 1 == T / 2) STACK_TL(1, 2);
    step(t - 1, sB, cB);
  }
  if (t == 0) step(0, sA, cA);
  STACK_TL(1, 3);
  SSTAMP_FLUSH(1, 0, wave == 0)
  store_step(0);
  mta_wait_vmem();
  __syncthreads();  // F
}

template <int H, int PREC>
__global__ __launch_bounds__((H / 16) * 128) void lstm_stack_bwd_kernel(StackBwdArgs a) {
  // one dynamic LDS block: the recurrence image (BwdSmem) or a weight-gradient staging image
  extern __shared__ __attribute__((aligned(16))) char dyn_lds[];
  const unsigned base = read_epoch_base(a.ctl, CTL_BWD_EPOCH, a.eshift);
  const int nrec = a.L * a.tr8;
  if ((int)blockIdx.x < nrec) {
    // producers of a hand-off always have lower block ids than their consumers (dispatch is in id order,
    // so every workgroup a spinning one waits for is already resident): top layer first here
    const int layer = a.L - 1 - blockIdx.x / a.tr8, tile = blockIdx.x % a.tr8;
    if (tile < a.ntiles) {
      const bool top = layer == a.L - 1, bottom = layer == 0;
      auto& sm = *reinterpret_cast<BwdSmem<H, PREC>*>(dyn_lds);
      if (top && bottom) stack_bwd_body<H, PREC, true, true, 1>(a, layer, tile, sm, base);
      else if (top) stack_bwd_body<H, PREC, true, false, 1>(a, layer, tile, sm, base);
      else if (a.L <= 2) {
        if (bottom) stack_bwd_body<H, PREC, false, true, 1>(a, layer, tile, sm, base);
        else stack_bwd_body<H, PREC, false, false, 1>(a, layer, tile, sm, base);
      } else {
        if (bottom) stack_bwd_body<H, PREC, false, true, 2>(a, layer, tile, sm, base);
        else stack_bwd_body<H, PREC, false, false, 2>(a, layer, tile, sm, base);
      }
    }
  } else {
    // fused weight gradient of (layer, time chunk, c' block), top layer and late chunks first (the order
    // in which the recurrence drains dG); waits until every tile of the layer has drained the chunk's steps
    const int idx = blockIdx.x - nrec;
    // layer-major, late chunks first (chunk-major order -- the order chunks become ready -- was slower at every batch
    // but B=1: B=8 bwd 175 -> 198 us, B=64 1,060 -> 1,203, profiles/r6_lstm_dec/r7g_probe.txt)
    const int layer = a.L - 1 - idx / a.wg_per_layer, rem = idx % a.wg_per_layer;
    const mta_wgrad::WgArgs& w = a.wg[layer];
    const int chunk = w.nchunks - 1 - rem / a.wg_nq, quarter = rem % a.wg_nq;
    const int t_lo = (int)((long)chunk * w.rows_per_chunk / a.Np);  // earliest step of the chunk's rows
    STACK_TLW(0);
    auto ready = [&]() {
      if (threadIdx.x < a.ntiles)
        wait_progress_far(a.dg_flags + FLAG_STRIDE * (layer * a.tr8 + threadIdx.x), base + (unsigned)(a.T - t_lo),
                          base, a.timeout, a.spin_limit);
      __syncthreads();
      STACK_TLW(1);
    };
    mta_wgrad::wgrad_body<PREC, H / 8, true>(w, chunk, quarter, dyn_lds, ready);
    STACK_TLW(2);
  }
  if (finish_launch(a.ctl, CTL_BWD_EPOCH, CTL_BWD_DONE, base, a.eshift) && a.dropout) {
    // fresh counter-hash masks for the next step (the graph needs no seed-update node)
    for (int l = 0; l < a.L; ++l) a.seeds[l] += 0x9E3779B97F4A7C15ull;
  }
  if ((int)blockIdx.x >= a.L * a.tr8) STACK_TLW(3);
}

template <int H, int PREC>
int launch_fwd(int fin, const StackFwdArgs& a, hipStream_t st) {
  const dim3 grid(a.main_blocks + (a.gather ? a.copy_blocks : 0)), block((H / 16) * 192);  // + batch-copy blocks
  const bool dec = a.dec != 0;
  if (fin == 3) {
    if (dec) lstm_stack_fwd_kernel<H, PREC, 3, true><<<grid, block, 0, st>>>(a);
    else lstm_stack_fwd_kernel<H, PREC, 3, false><<<grid, block, 0, st>>>(a);
  } else if (fin == 5) {
    if (dec) lstm_stack_fwd_kernel<H, PREC, 5, true><<<grid, block, 0, st>>>(a);
    else lstm_stack_fwd_kernel<H, PREC, 5, false><<<grid, block, 0, st>>>(a);
  } else {
    return -1;
  }
  return 0;
}

template <int H>
int dispatch_fwd(int prec, int fin, const StackFwdArgs& a, hipStream_t st) {
  if (prec == PREC_F32) return launch_fwd<H, PREC_F32>(fin, a, st);
  if (prec == PREC_BF16X3) return launch_fwd<H, PREC_BF16X3>(fin, a, st);
  if (prec == PREC_F16X2) return launch_fwd<H, PREC_F16X2>(fin, a, st);
  return launch_fwd<H, PREC_BF16>(fin, a, st);
}

template <int H, int PREC>
int launch_bwd(const StackBwdArgs& a, size_t lds, hipStream_t st) {
  const dim3 grid(a.L * a.tr8 + a.L * a.wg_per_layer), block((H / 16) * 128);  // recurrent + gradient waves
  lds = lds > sizeof(BwdSmem<H, PREC>) ? lds : sizeof(BwdSmem<H, PREC>);
  if (lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_stack_bwd_kernel<H, PREC>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -3;
  lstm_stack_bwd_kernel<H, PREC><<<grid, block, lds, st>>>(a);
  return 0;
}

template <int H>
int dispatch_bwd(int prec, const StackBwdArgs& a, size_t wg_lds, hipStream_t st) {
  if (prec == PREC_F32) return launch_bwd<H, PREC_F32>(a, wg_lds, st);
  // PREC_F16X2 is a forward mode: the backward products stay bf16x3 (gradients need bf16's exponent range)
  if (prec == PREC_BF16X3 || prec == PREC_F16X2) return launch_bwd<H, PREC_BF16X3>(a, wg_lds, st);
  return launch_bwd<H, PREC_BF16>(a, wg_lds, st);
}

unsigned spin_limit() {
  static const unsigned v = [] {
    const char* e = getenv("MTA_LSTM_SPIN_LIMIT");
    return e && atol(e) > 0 ? (unsigned)atol(e) : SPIN_LIMIT;
  }();
  return v;
}

}  // namespace

// flags (zero-initialised once, then never reset): [3][MAXL][tr8] progress words (forward, backward dX,
// backward dG; FLAG_STRIDE apart) + CTL_WORDS control words (timeout, per-direction epoch + arrival counter).
extern "C" int mta_lstm_stack_epoch_shift(int T) { return epoch_shift(T); }

// flags layout: [3][MAXL][tr8] progress words (FLAG_STRIDE apart) | [2][MAXL][tr8] XCC ids (fwd, bwd) | CTL_WORDS
extern "C" long mta_lstm_stack_flag_words(int Np) {
  const int tr8 = (Np / S + 7) / 8 * 8;
  return 3L * FLAG_STRIDE * MAXL * tr8 + 2L * MAXL * tr8 + CTL_WORDS;
}
namespace {
unsigned* ctl_words(unsigned* flags, int tr8) { return flags + 3L * FLAG_STRIDE * MAXL * tr8 + 2L * MAXL * tr8; }
unsigned* xcc_words(unsigned* flags, int tr8, int dir) { return flags + 3L * FLAG_STRIDE * MAXL * tr8 + (long)dir * MAXL * tr8; }
int xcd_local_enabled() {
  static const int v = [] {
    const char* e = getenv("MTA_LSTM_XCD_LOCAL");
    return e && atoi(e) == 0 ? 0 : 1;
  }();
  return v;
}
}  // namespace

// gather (nullable): x is then the static batch buffer the launch fills (layer 0 reads the dataset directly)
extern "C" int mta_lstm_stack_fwd_g(int H, int prec, int L, int fin, const float* x, const float* const* w_ih,
                                    const float* const* w_hh, const float* const* b_ih, const float* const* b_hh,
                                    float* const* hseq, float* const* xdrop, uint32_t* const* mask,
                                    float* const* stash, const uint64_t* seeds, float drop_p, unsigned* flags, int N,
                                    int Np, int T, const MtaBatchGather* gather, unsigned long long* gran,
                                    int decoupled, hipStream_t st) {
  if (L < 1 || L > MAXL || Np % S || N > Np || N < 1 || (H != 32 && H != 64)) return -1;
  StackFwdArgs a{};
  a.x = x;
  // decoupled form: L = 1 needs no hand-off buffer; deeper stacks take gran = (L - 1) x (T, Np, H) granules
  if (decoupled && L > 1 && !gran) return -5;
  if (decoupled && L > 1)
    for (int l = 1; l < L; ++l) a.gran[l] = gran + (size_t)(l - 1) * T * Np * H;
  a.dec = decoupled ? 1 : 0;
  if (gather) {
    if (gather->B < 1 || N % gather->B || gather->nt < 1 || gather->nt > 4 || gather->src[0] == nullptr ||
        gather->row[0] != (long)(N / gather->B) * T * fin)
      return -4;
    a.gather = 1;
    a.g = *gather;
  }
  for (int l = 0; l < L; ++l) {
    a.w_ih[l] = w_ih[l];
    a.w_hh[l] = w_hh[l];
    a.b_ih[l] = b_ih[l];
    a.b_hh[l] = b_hh[l];
    a.hseq[l] = hseq[l];
    a.xdrop[l] = xdrop ? xdrop[l] : nullptr;
    a.mask[l] = mask ? mask[l] : nullptr;
    if (a.xdrop[l] && !a.mask[l]) return -2;  // the backward reads the keep bytes
    a.stash[l] = stash ? stash[l] : nullptr;
  }
  a.seeds = seeds;
  a.drop_p = drop_p;
  a.N = N;
  a.Np = Np;
  a.T = T;
  a.L = L;
  a.ntiles = Np / S;
  a.tr8 = (a.ntiles + 7) / 8 * 8;  // tile i of every layer gets the same block id modulo 8
  a.eshift = epoch_shift(T);
  if (T + 8 >= (1 << a.eshift)) return -1;
  a.flags = flags;
  a.ctl = ctl_words(flags, a.tr8);
  a.xcc = xcc_words(flags, a.tr8, 0);
  a.timeout = a.ctl + CTL_TIMEOUT;
  a.spin_limit = spin_limit();
  a.main_blocks = a.L * a.tr8;
  a.copy_blocks = 16;
  // the partner XCC exchange waits for the consumer workgroup to start: only with the whole grid co-resident
  a.xcd_local = xcd_local_enabled() && a.main_blocks + a.copy_blocks <= 256;
  if (H == 32) return dispatch_fwd<32>(prec, fin, a, st);
  return dispatch_fwd<64>(prec, fin, a, st);
}

extern "C" int mta_lstm_stack_fwd(int H, int prec, int L, int fin, const float* x, const float* const* w_ih,
                                  const float* const* w_hh, const float* const* b_ih, const float* const* b_hh,
                                  float* const* hseq, float* const* xdrop, uint32_t* const* mask,
                                  float* const* stash, const uint64_t* seeds, float drop_p, unsigned* flags, int N,
                                  int Np, int T, unsigned long long* gran, int decoupled, hipStream_t st) {
  return mta_lstm_stack_fwd_g(H, prec, L, fin, x, w_ih, w_hh, b_ih, b_hh, hseq, xdrop, mask, stash, seeds, drop_p,
                              flags, N, Np, T, nullptr, gran, decoupled, st);
}

// Weight gradients are fused when g_whh is given: inp[0] = x (N, T, fin) batch-first, inp[l >= 1] = the layer's
// (dropped-out) input sequence (T, Np, H); the gradients accumulate into g_* (the flat gradient buffer).
// rows of one fused weight-gradient workgroup's chunk above which the chunk is split in two (B >= 8 windows:
// Np >= 800).  Two parts beat three or more at every measured batch -- more parts mean more partial atomics and
// more spinning workgroups (profiles/r5_lstm_wgrad_row_split.txt)
constexpr int WG_FUSED_SPLIT_ROWS = 512;
// 65-128-row chunks (B = 1: one step of Np = 112 rows) are split in two as well: the chunk of step 0 -- the
// backward's tail -- is then two 2-slice workgroups instead of one 4-slice one (body 11 -> 7.9 us; L=2 backward
// 89.3 -> 86.2 us, L=4 129.3 -> 127.5, profiles/r6_lstm_dec/r7a_probe.txt)
constexpr int WG_SMALL_SPLIT_MIN = 2 * mta_wgrad::WG_KS, WG_SMALL_SPLIT_MAX = 4 * mta_wgrad::WG_KS;

extern "C" int mta_lstm_stack_bwd(int H, int prec, int L, int fin, const float* const* stash, const float* const* w_hh,
                                  const float* const* w_ih, const float* dh_last, float* const* dG, float* const* dX,
                                  const float* const* hseq, const float* const* inp, float* const* g_wih,
                                  float* const* g_whh, float* const* g_bih, float* const* g_bhh,
                                  const uint32_t* const* mask, float* const* part, uint64_t* seeds, float drop_p,
                                  int dropout, unsigned* flags, int N, int Np, int T, int form, hipStream_t st) {
  if (L < 1 || L > MAXL || Np % S || N > Np || N < 1 || (H != 32 && H != 64) || T + 8 >= (1 << MAX_EPOCH_SHIFT)) return -1;
  if (prec == PREC_F16X2) prec = PREC_BF16X3;  // a forward mode: backward products in bf16x3
  StackBwdArgs a{};
  for (int l = 0; l < L; ++l) {
    a.stash[l] = stash[l];
    a.w_hh[l] = w_hh[l];
    a.w_ih[l] = w_ih[l];
    a.dG[l] = dG[l];
    a.dX[l] = dX ? dX[l] : nullptr;
    a.mask[l] = mask ? mask[l] : nullptr;
    if (dropout && l > 0 && !a.mask[l]) return -2;
  }
  a.dh_last = dh_last;
  // form: the dX hand-off, 0 = fp32 rows + progress words (the tagged-granule form 1 was measured slower at every
  // depth and removed, profiles/r6_lstm_decoupled.txt)
  if (form != 0) return -1;
  a.seeds = seeds;
  a.drop_p = drop_p;
  a.dropout = dropout;
  a.N = N;
  a.Np = Np;
  a.T = T;
  a.L = L;
  a.ntiles = Np / S;
  a.tr8 = (a.ntiles + 7) / 8 * 8;
  a.eshift = epoch_shift(T);
  a.flags = flags + FLAG_STRIDE * MAXL * a.tr8;
  a.dg_flags = flags + 2 * FLAG_STRIDE * MAXL * a.tr8;
  a.ctl = ctl_words(flags, a.tr8);
  a.timeout = a.ctl + CTL_TIMEOUT;
  a.spin_limit = spin_limit();
  size_t wg_lds = 0;
  if (g_whh) {
    // NWAVES = 2 H / 16 waves per workgroup -> CQ = 16 NWAVES gate columns, 4H / CQ = 2 blocks per chunk
    const int nwaves = H / 8, cq = 16 * nwaves;
    const int tc = mta_wgrad::wg_time_chunk(T, true);
    a.wg_nq = 4 * H / cq;
    // large batches: split a time chunk's rows over two workgroups, so the chunk of the earliest steps
    // (drained last) is not a serial tail of tc * Np rows behind the recurrence
    int rpc = tc * Np;
    if (!part && (rpc > WG_FUSED_SPLIT_ROWS || (rpc > WG_SMALL_SPLIT_MIN && rpc <= WG_SMALL_SPLIT_MAX)))
      // (deterministic mode keeps tc-step chunks: its partials are sized so)
      rpc = ((rpc + 1) / 2 + mta_wgrad::WG_KS - 1) / mta_wgrad::WG_KS * mta_wgrad::WG_KS;
    for (int l = 0; l < L; ++l) {
      mta_wgrad::WgArgs& w = a.wg[l];
      w.dG = dG[l];
      w.hseq = hseq[l];
      w.inp = inp[l];
      w.inp_batch_first = l == 0;
      w.N = N;
      w.Np = Np;
      w.T = T;
      w.H = H;
      w.F = l == 0 ? fin : H;
      w.FP = (w.F + 15) / 16 * 16;
      w.rows_per_chunk = rpc;
      w.nchunks = (T * Np + rpc - 1) / rpc;
      w.g_wih = g_wih[l];
      w.g_whh = g_whh[l];
      w.g_bih = g_bih[l];
      w.g_bhh = g_bhh[l];
      w.part = part ? part[l] : nullptr;
      const int NB = H + w.FP;
      if (NB / 16 > 16 || cq + NB > mta_wgrad::WG_MAX_UNITS_PER_THREAD * 64 * nwaves) return -1;
      size_t bytes;
      if (prec == PREC_F32) {
        w.lo_off = 0;
        bytes = (size_t)(cq + NB) * mta_wgrad::WgImg<PREC_F32>::RS * 4;
      } else {
        w.lo_off = (cq + NB) * mta_wgrad::WgImg<PREC_BF16>::RS;
        bytes = (size_t)w.lo_off * 2 * (prec == PREC_BF16X3 ? 2 : 1);
      }
      wg_lds = bytes > wg_lds ? bytes : wg_lds;
    }
    a.wg_per_layer = a.wg[0].nchunks * a.wg_nq;
  }
  const int rc = H == 32 ? dispatch_bwd<32>(prec, a, wg_lds, st) : dispatch_bwd<64>(prec, a, wg_lds, st);
  if (rc == 0 && g_whh && part) {
    // deterministic mode: the fused workgroups wrote per-chunk partials; add them in chunk order
    for (int l = 0; l < L; ++l)
      if (a.wg[l].part)
        mta_wgrad::wgrad_reduce_kernel<<<(int)((mta_wgrad::wg_part_elems(H, a.wg[l].F) + 255) / 256), 256, 0, st>>>(
            a.wg[l]);
  }
  return rc;
}
