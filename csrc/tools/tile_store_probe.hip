// Diagnostic probe (not part of the extension): chip-wide store bandwidth of a GEMM epilogue's output pattern.
// 256 workgroups x 512 threads each write one 256 x 256 f32 tile of a [R][ldc] matrix (as the 256 x 256 GEMM's
// epilogue: wave (wm, wn) owns rows 128 wm .., cols 64 wn ..; one 16-B store per lane covers 4 rows x 256 B), against
// the same bytes written as one contiguous 256-KB block per workgroup.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 csrc/tools/tile_store_probe.hip -o tools_bin/tile_store_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

template <int MODE>
__global__ __launch_bounds__(512) void store_kernel(float* out, int ldc, int tiles_x) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 2, wn = wave & 3;
  const int bx = blockIdx.x % tiles_x, by = blockIdx.x / tiles_x;
  const float4 v = make_float4(1.f * lane, 2.f, 3.f, 4.f);
  if (MODE == 0) {  // GEMM tile pattern
    const int col = bx * 256 + wn * 64 + 4 * (lane & 15);
    for (int q = 0; q < 32; ++q) {
      const int row = by * 256 + wm * 128 + 4 * q + (lane >> 4);
      *reinterpret_cast<float4*>(out + (size_t)row * ldc + col) = v;
    }
  } else if (MODE == 1) {  // contiguous 256 KB per workgroup
    float* base = out + (size_t)blockIdx.x * 65536;
    for (int q = 0; q < 32; ++q) *reinterpret_cast<float4*>(base + ((size_t)q * 512 + threadIdx.x) * 4) = v;
  } else {  // GEMM tile pattern, nontemporal
    const int col = bx * 256 + wn * 64 + 4 * (lane & 15);
    for (int q = 0; q < 32; ++q) {
      const int row = by * 256 + wm * 128 + 4 * q + (lane >> 4);
      typedef float f4 __attribute__((ext_vector_type(4)));
      const f4 w = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(w, reinterpret_cast<f4*>(out + (size_t)row * ldc + col));
    }
  }
}

int main() {
  const int R = 4096, C = 4096;
  float* out;
  CK(hipMalloc(&out, (size_t)R * C * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 3; ++mode) {
    std::vector<float> ts;
    for (int r = 0; r < 23; ++r) {
      CK(hipEventRecord(e0, 0));
      if (mode == 0) store_kernel<0><<<256, 512>>>(out, C, 16);
      else if (mode == 1) store_kernel<1><<<256, 512>>>(out, C, 16);
      else store_kernel<2><<<256, 512>>>(out, C, 16);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    printf("%-22s %8.2f us  %6.2f TB/s\n", mode == 0 ? "tile pattern" : mode == 1 ? "contiguous per WG" : "tile pattern nt", us,
           (double)R * C * 4 / (us * 1e-6) / 1e12);
  }
  return 0;
}
