// All-reduce over xGMI peer memory for the DDP gradient buckets of one node (SURVEY §2.6 M2 / §5 "Distributed").
//
// Every rank owns one fine-grained (cross-device coherent) comm buffer, exported by IPC and mapped by every
// peer.  A bucket is a range [off, off + n) of the flat gradient; each bucket owns a CHANNEL (its own epoch,
// arrival counters and flag rows), so the buckets of one step can be reduced concurrently, each launched on a
// side stream as soon as the backward has produced it (ops/extras.py, parallel/ddp.py).
//
//   comm buffer: inbox[2 parity][world][cap] | gather[2 parity][cap] | flags[channels][2 phases][world][32 words]
//
// One launch per bucket, step epoch e of its channel (device-resident counter: graph capturable), parity e & 1.
//   ONE-SHOT (small buckets: latency-bound, one hop):
//     push   : every workgroup writes its slice of the bucket into slot `rank` of EVERY rank's inbox (remote
//              stores over xGMI, all 7 links in parallel), system-scope release;
//     signal : the last local workgroup to arrive stores flag[ch][0][rank] = e into every rank's flag rows;
//     wait   : every workgroup polls its own flag rows until all `world` flags reach e (bounded: a give-up
//              counts in the timeout word the host checks, so the grid always drains), system-scope acquire;
//     reduce : sum of the `world` slots in rank order (identical on every rank: replicas stay bit-identical).
//   TWO-SHOT (large buckets: each rank sends 2 (N-1)/N of the bucket instead of N-1 copies of it):
//     reduce-scatter: chunk c of the bucket goes to rank c's inbox slot `rank`; signal / wait (phase 0);
//                     rank r sums its chunk's `world` slots in rank order and pushes the sum into the gather
//                     region of every rank; signal / wait (phase 1);
//     all-gather    : copy the gather region of the bucket back into the gradient.
// Double buffering by parity is enough: a rank only starts call e+2 of a channel after every peer signalled
// phase 0 of e+1, i.e. after every peer finished call e.  Flags compare with a wrap-safe ">=".
// Workgroups per launch stay <= XG_BIG_BLOCKS so the grid is co-resident beside a concurrent backward kernel (a
// workgroup waits for the arrival of its rank's others: a non-resident one would stall it until the bound).
#include <cstdlib>

#include "common.h"

namespace {

constexpr int XG_MAX = 8;
constexpr int XG_TPB = 256;
constexpr int XG_SMALL_BLOCKS = 32, XG_BIG_BLOCKS = 128;  // grid caps (<= 8 MB / larger buckets)
constexpr int XG_FLAG_STRIDE = 32;  // words: one 128-byte line per flag
constexpr int XG_MAX_CHANNELS = 64;
// ctl (local device memory): per channel [epoch, arrive phase 0, arrive phase 1, pad] in one 128-byte line, then
// the shared timeout word
constexpr int XG_CTL_STRIDE = 32;
constexpr int XG_TIMEOUT = XG_MAX_CHANNELS * XG_CTL_STRIDE;
constexpr int XG_CTL_WORDS = XG_TIMEOUT + 32;
constexpr unsigned XG_SPIN_LIMIT = 1u << 28;  // ~16 s of polls: far beyond any step skew

struct XgmiArgs {
  float4* grad;                // the bucket (n4 float4) in the local gradient
  long n4, off4, cap4, chunk4;
  float4* peer_inbox[XG_MAX];  // every rank's inbox region (own included), mapped in this process
  float4* peer_gather[XG_MAX];
  unsigned* peer_flags[XG_MAX];  // this channel's flag rows in every rank's buffer: [2 phases][world][32]
  unsigned* ctl;               // this channel's ctl line
  unsigned* timeout;
  // clip-norm partials of the reduced bucket (nullable): workgroup b writes the sum of squares of the values it
  // stored into the gradient to sq[b] (the fused optimizer sums them instead of re-reading the buffer)
  float* sq;
  int rank, world, twoshot;
};

__device__ __forceinline__ float f4sq(float4 v) { return fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, v.w * v.w))); }

__device__ __forceinline__ float4 f4add(float4 s, float4 v) {
  s.x += v.x;
  s.y += v.y;
  s.z += v.z;
  s.w += v.w;
  return s;
}

// every workgroup arrives on the channel's phase counter after a system release of its pushes; the last one
// re-arms the counter and signals `epoch` to every rank's flag row [phase][rank]; then every workgroup waits for
// all `world` flags of the phase and acquires
__device__ void xg_signal_wait(const XgmiArgs& a, int phase, unsigned epoch) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this workgroup's remote stores first
  __syncthreads();
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.ctl + 1 + phase, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last && threadIdx.x < a.world) {
    if (threadIdx.x == 0) {
      __hip_atomic_store(a.ctl + 1 + phase, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // every workgroup read the epoch before arriving on phase 0: the last arriver advances it
      if (phase == 0) __hip_atomic_store(a.ctl, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __hip_atomic_store(a.peer_flags[threadIdx.x] + (phase * a.world + a.rank) * XG_FLAG_STRIDE, epoch,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x < a.world) {
    unsigned* f = a.peer_flags[a.rank] + (phase * a.world + threadIdx.x) * XG_FLAG_STRIDE;
    unsigned spins = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > XG_SPIN_LIMIT) {
        __hip_atomic_fetch_add(a.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the peers' pushes are visible
}

__global__ __launch_bounds__(XG_TPB) void xgmi_allreduce_kernel(XgmiArgs a) {
  // every workgroup reads the epoch before arriving on phase 0, whose last arriver advances it
  const unsigned epoch = __hip_atomic_load(a.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const long par = epoch & 1;
  const long stride = (long)gridDim.x * XG_TPB, first = (long)blockIdx.x * XG_TPB + threadIdx.x;
  const float4* my_inbox = a.peer_inbox[a.rank] + par * a.world * a.cap4 + a.off4;
  float sq = 0.f;  // squares of every value this workgroup stores into the gradient (its last pass over them)
  if (!a.twoshot) {
    for (long i = first; i < a.n4; i += stride) {
      const float4 v = a.grad[i];
      for (int p = 0; p < a.world; ++p) a.peer_inbox[p][(par * a.world + a.rank) * a.cap4 + a.off4 + i] = v;
    }
    xg_signal_wait(a, 0, epoch);
    for (long i = first; i < a.n4; i += stride) {
      float4 s = my_inbox[i];
      for (int p = 1; p < a.world; ++p) s = f4add(s, my_inbox[(long)p * a.cap4 + i]);
      a.grad[i] = s;
      sq += f4sq(s);
    }
  } else {
    // reduce-scatter: element i belongs to chunk i / chunk4 (owner rank)
    for (long i = first; i < a.n4; i += stride) {
      const int p = (int)(i / a.chunk4);
      a.peer_inbox[p][(par * a.world + a.rank) * a.cap4 + a.off4 + i] = a.grad[i];
    }
    xg_signal_wait(a, 0, epoch);
    const long c0 = (long)a.rank * a.chunk4, c1 = c0 + a.chunk4 < a.n4 ? c0 + a.chunk4 : a.n4;
    for (long i = c0 + first; i < c1; i += stride) {
      float4 s = my_inbox[i];
      for (int p = 1; p < a.world; ++p) s = f4add(s, my_inbox[(long)p * a.cap4 + i]);
      for (int p = 0; p < a.world; ++p) a.peer_gather[p][par * a.cap4 + a.off4 + i] = s;
    }
    xg_signal_wait(a, 1, epoch);
    const float4* g = a.peer_gather[a.rank] + par * a.cap4 + a.off4;
    for (long i = first; i < a.n4; i += stride) {
      const float4 v = g[i];
      a.grad[i] = v;
      sq += f4sq(v);
    }
  }
  if (a.sq) {
    __shared__ float scr[XG_TPB / 64];
    sq = block_sum(sq, scr);  // the same workgroup -> slot and summation order every step: deterministic
    if (threadIdx.x == 0) a.sq[blockIdx.x] = sq;
  }
}

struct Layout {
  long inbox, gather, flags, total;
};
Layout layout(int world, long cap, int channels) {
  Layout l;
  l.inbox = 0;
  l.gather = 2L * world * cap * 4;
  l.flags = (l.gather + 2L * cap * 4 + 127) / 128 * 128;
  l.total = l.flags + (long)channels * 2 * world * XG_FLAG_STRIDE * 4;
  return l;
}

}  // namespace

extern "C" {

// comm buffer of one rank: fine-grained device memory (coherent for peer access), zeroed
int mta_xgmi_alloc(long bytes, void** out) {
  if (hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocFinegrained) != hipSuccess) return -1;
  if (hipMemset(*out, 0, (size_t)bytes) != hipSuccess) return -2;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}

int mta_xgmi_free(void* p) { return hipFree(p) == hipSuccess ? 0 : -1; }

int mta_xgmi_ipc_handle(void* p, unsigned char* out64) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) return -1;
  static_assert(sizeof(h) <= 64, "IPC handle larger than 64 bytes");
  for (size_t i = 0; i < sizeof(h); ++i) out64[i] = reinterpret_cast<const unsigned char*>(&h)[i];
  return (int)sizeof(h);
}

int mta_xgmi_ipc_open(const unsigned char* in64, void** out) {
  hipIpcMemHandle_t h;
  for (size_t i = 0; i < sizeof(h); ++i) reinterpret_cast<unsigned char*>(&h)[i] = in64[i];
  return hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? 0 : -1;
}

int mta_xgmi_ipc_close(void* p) { return hipIpcCloseMemHandle(p) == hipSuccess ? 0 : -1; }

long mta_xgmi_buffer_bytes(int world, long cap, int channels) { return layout(world, cap, channels).total; }

int mta_xgmi_ctl_words() { return XG_CTL_WORDS; }
int mta_xgmi_max_channels() { return XG_MAX_CHANNELS; }
int mta_xgmi_timeout_word() { return XG_TIMEOUT; }

// grad: the bucket's n floats (n % 4 == 0) at flat offset `off` (off % 4 == 0, off + n <= cap); bufs[p]: rank p's
// comm buffer as mapped here (own included); twoshot: reduce-scatter + all-gather instead of one-shot
int mta_xgmi_max_blocks() { return XG_BIG_BLOCKS; }

// sq (nullable): mta_xgmi_max_blocks() floats of clip-norm partials of this bucket (zero where no workgroup ran)
int mta_xgmi_allreduce(float* grad, long n, long off, long cap, int channel, int channels, int twoshot,
                       void* const* bufs, int rank, int world, unsigned* ctl, float* sq, hipStream_t st) {
  if (world < 1 || world > XG_MAX || rank < 0 || rank >= world || n % 4 || off % 4 || cap % 4 || off + n > cap ||
      channel < 0 || channel >= channels || channels > XG_MAX_CHANNELS || n <= 0)
    return -1;
  const Layout l = layout(world, cap, channels);
  XgmiArgs a{};
  a.grad = reinterpret_cast<float4*>(grad);
  a.n4 = n / 4;
  a.off4 = off / 4;
  a.cap4 = cap / 4;
  a.chunk4 = (a.n4 + world - 1) / world;
  for (int p = 0; p < world; ++p) {
    char* b = reinterpret_cast<char*>(bufs[p]);
    a.peer_inbox[p] = reinterpret_cast<float4*>(b + l.inbox);
    a.peer_gather[p] = reinterpret_cast<float4*>(b + l.gather);
    a.peer_flags[p] = reinterpret_cast<unsigned*>(b + l.flags) + (long)channel * 2 * world * XG_FLAG_STRIDE;
  }
  a.ctl = ctl + channel * XG_CTL_STRIDE;
  a.timeout = ctl + XG_TIMEOUT;
  a.rank = rank;
  a.world = world;
  a.twoshot = twoshot ? 1 : 0;
  a.sq = sq;
  // grid cap by bucket size (profiles/r4_xgmi_local.txt, 2 processes on one GPU): up to 8 MB the flag protocol
  // dominates and fewer workgroups are faster (3.2 MB one-shot: 29 us at 32, 31 at 64, 35 at 128); a 52 MB bucket
  // is bandwidth-bound (547 / 330 / 233 / 224 us at 32 / 64 / 128 / 256).  At most 256 (one per CU: every
  // workgroup waits for its rank's others, so the grid must be co-resident beside a concurrent backward).
  const long max_blocks = n * 4L > (8L << 20) ? XG_BIG_BLOCKS : XG_SMALL_BLOCKS;
  long blocks = (a.n4 + XG_TPB * 8 - 1) / (XG_TPB * 8);
  blocks = blocks < 1 ? 1 : blocks > max_blocks ? max_blocks : blocks;
  xgmi_allreduce_kernel<<<(int)blocks, XG_TPB, 0, st>>>(a);
  return 0;
}

}  // extern "C"
