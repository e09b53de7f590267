// One-shot all-reduce over xGMI peer memory (the DDP gradient sum of one node, SURVEY §2.6 M2 / §5
// "Distributed"): a single kernel per rank replaces the RCCL ring for the small flat gradient buckets of this
// workload (204 KB for model=small), where a ring's 2 (N-1) latency-bound hops dominate.
//
// Every rank owns one fine-grained (cross-device coherent) comm buffer, exported by IPC and mapped by every
// peer:  data[2 parity][world slots][cap floats] | flags[world][32 words].  One launch, step epoch e
// (device-resident counter: graph capturable), parity e & 1:
//   push   : every workgroup writes its slice of the local gradient into slot `rank` of EVERY rank's buffer
//            (remote stores over xGMI; one link per peer, all links in parallel), system-scope release fence;
//   signal : the last workgroup to arrive (local counter) stores flag[rank] = e into every rank's flag row;
//   wait   : every workgroup polls its own flag row until all `world` flags reach e (bounded: a give-up counts
//            in the timeout word the host checks, so the grid always drains), system-scope acquire fence;
//   reduce : every workgroup sums the `world` slots of its slice in rank order (identical on every rank:
//            the replicas stay bit-identical) into the local gradient.
// Double buffering by parity is enough: a rank can only start step e+2 after every peer has signalled step
// e+1, i.e. after every peer finished reading step e.  Flags are compared with a wrap-safe ">=" (a fast peer
// may already have signalled e+1 while this rank waits for e).
#include "common.h"

namespace {

constexpr int XG_MAX = 8;
constexpr int XG_TPB = 256;
constexpr int XG_FLAG_STRIDE = 32;  // words: one 128-byte line per flag
enum { XG_EPOCH = 0, XG_ARRIVE = 32, XG_TIMEOUT = 64, XG_CTL_WORDS = 96 };
constexpr unsigned XG_SPIN_LIMIT = 1u << 28;  // ~16 s of polls: far beyond any step skew

struct XgmiArgs {
  float4* grad;
  long n4, cap4;
  float4* peer_data[XG_MAX];   // every rank's data region (own included), mapped in this process
  unsigned* peer_flags[XG_MAX];
  float4* my_data;
  unsigned* my_flags;
  unsigned* ctl;               // local device memory: epoch, arrival counter, timeout count
  int rank, world;
};

__global__ __launch_bounds__(XG_TPB) void xgmi_allreduce_kernel(XgmiArgs a) {
  const unsigned epoch = __hip_atomic_load(a.ctl + XG_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int parity = epoch & 1;
  const long stride = (long)gridDim.x * XG_TPB;
  // ---- push ----
  for (long i = (long)blockIdx.x * XG_TPB + threadIdx.x; i < a.n4; i += stride) {
    const float4 v = a.grad[i];
    for (int p = 0; p < a.world; ++p) a.peer_data[p][((long)parity * a.world + a.rank) * a.cap4 + i] = v;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the remote stores are visible first
  __syncthreads();
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.ctl + XG_ARRIVE, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  // ---- signal (last arriver: every workgroup's pushes were released before its arrival) ----
  if (s_last && threadIdx.x < a.world) {
    if (threadIdx.x == 0) {
      __hip_atomic_store(a.ctl + XG_ARRIVE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.ctl + XG_EPOCH, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __hip_atomic_store(a.peer_flags[threadIdx.x] + a.rank * XG_FLAG_STRIDE, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // ---- wait ----
  if (threadIdx.x < a.world) {
    unsigned* f = a.my_flags + threadIdx.x * XG_FLAG_STRIDE;
    unsigned spins = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > XG_SPIN_LIMIT) {
        __hip_atomic_fetch_add(a.ctl + XG_TIMEOUT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the peers' pushes are visible
  // ---- reduce (rank order: bit-identical on every rank) ----
  const float4* base = a.my_data + (long)parity * a.world * a.cap4;
  for (long i = (long)blockIdx.x * XG_TPB + threadIdx.x; i < a.n4; i += stride) {
    float4 s = base[i];
    for (int p = 1; p < a.world; ++p) {
      const float4 v = base[(long)p * a.cap4 + i];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    a.grad[i] = s;
  }
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

long mta_xgmi_layout(int world, long cap, long* flags_off) {
  // data: 2 x world x cap floats, then the flag rows (128-byte aligned)
  const long data = 2L * world * cap * 4;
  *flags_off = (data + 127) / 128 * 128;
  return *flags_off + (long)world * XG_FLAG_STRIDE * 4;
}

int mta_xgmi_ctl_words() { return XG_CTL_WORDS; }

// grad: n floats (n % 4 == 0, n <= cap); bufs[p]: rank p's comm buffer as mapped here (own included)
int mta_xgmi_allreduce(float* grad, long n, long cap, void* const* bufs, int rank, int world, unsigned* ctl,
                       hipStream_t st) {
  if (world < 1 || world > XG_MAX || rank < 0 || rank >= world || n % 4 || cap % 4 || n > cap) return -1;
  XgmiArgs a{};
  long flags_off = 0;
  mta_xgmi_layout(world, cap, &flags_off);
  a.grad = reinterpret_cast<float4*>(grad);
  a.n4 = n / 4;
  a.cap4 = cap / 4;
  for (int p = 0; p < world; ++p) {
    a.peer_data[p] = reinterpret_cast<float4*>(bufs[p]);
    a.peer_flags[p] = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(bufs[p]) + flags_off);
  }
  a.my_data = a.peer_data[rank];
  a.my_flags = a.peer_flags[rank];
  a.ctl = ctl;
  a.rank = rank;
  a.world = world;
  long blocks = (a.n4 + XG_TPB * 4 - 1) / (XG_TPB * 4);
  blocks = blocks < 1 ? 1 : blocks > 256 ? 256 : blocks;  // <= one per CU: all co-resident (the wait)
  xgmi_allreduce_kernel<<<(int)blocks, XG_TPB, 0, st>>>(a);
  return 0;
}

}  // extern "C"
