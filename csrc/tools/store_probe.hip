// Diagnostic probe (not part of the extension): per-CU vector-store throughput on gfx950, the resource the
// pipelined LSTM forward is suspected to be bound by (csrc/lstm_stack.hip stores ~29 KB per step per workgroup).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc csrc/tools/store_probe.hip -o tools_bin/store_probe
//   ./tools_bin/store_probe
// Each workgroup (W waves) issues R rounds of one 16-byte store per lane (1 KB per wave-instruction, contiguous),
// plain or write-through (sc1), into its own region; reports bytes per shader cycle per workgroup (s_memtime).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);           \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void store_kernel(float* out, int rounds, long region_floats, unsigned long long* cyc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  float* base = out + (size_t)blockIdx.x * region_floats;
  f32x4 v = {1.f * lane, 2.f, 3.f, 4.f};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < rounds; ++r) {
    float* p = base + ((size_t)(r * nw + wave) * 64 + lane) * 4;
    if (MODE == 0) {
      *reinterpret_cast<f32x4*>(p) = v;
    } else {
      asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
    }
    v.x += 1.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int rounds = 256;
  const long region = (long)rounds * 16 * 64 * 4;  // floats per workgroup (16 waves max)
  float* out;
  unsigned long long* cyc;
  const int max_blocks = 256;
  CK(hipMalloc(&out, (size_t)region * max_blocks * 4));
  CK(hipMalloc(&cyc, max_blocks * 8));
  unsigned long long hc[max_blocks];
  for (int mode = 0; mode < 2; ++mode)
    for (int blocks : {1, 14, 128})
      for (int waves : {4, 8, 12}) {
        for (int rep = 0; rep < 3; ++rep) {
          if (mode == 0) store_kernel<0><<<blocks, waves * 64>>>(out, rounds, region, cyc);
          else store_kernel<1><<<blocks, waves * 64>>>(out, rounds, region, cyc);
        }
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hc, cyc, blocks * 8, hipMemcpyDeviceToHost));
        double avg = 0;
        for (int b = 0; b < blocks; ++b) avg += (double)hc[b] / blocks;
        const double bytes = (double)rounds * waves * 1024;
        printf("%-5s blocks=%3d waves=%2d: %8.0f cycles for %6.0f KB per workgroup = %5.1f B/cycle/CU\n",
               mode ? "sc1" : "plain", blocks, waves, avg, bytes / 1024, bytes / avg);
      }
  return 0;
}
