// Diagnostic probe (not part of the extension): the 256 x 256 LDS-DMA GEMM of csrc/gemm.hip on one shape, timed, and
// (built with -DMTA_STAMPS) the s_memtime split of its main loop per wave.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc [-DMTA_STAMPS] \
//         csrc/tools/gemm_probe.hip -o tools_bin/gemm_probe
//   ./tools_bin/gemm_probe M N K mode
#include "../gemm.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

// the extension links optim.hip's zero-fill; the probe never requests a gradient-producer overwrite
extern "C" void mta_zero_bytes(void*, long, hipStream_t) {}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);           \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void fill_kernel(__bf16* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 0x9E3779B1u ^ seed;
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    p[i] = (__bf16)((float)(x & 0xFFFF) / 32768.f - 1.f);
  }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096;
  const int K = argc > 3 ? atoi(argv[3]) : 4096, mode = argc > 4 ? atoi(argv[4]) : 0;
  const int epi = argc > 5 ? atoi(argv[5]) : 0;  // 1: the MLP forward epilogue (bias + GELU, bf16 pre-activation)
  const int ksplit = argc > 6 ? atoi(argv[6]) : 1;  // split-K
  if (argc > 7) mta_gemm_set_big(atoi(argv[7]));      // -1 default, 0 off, 1 on
  __bf16 *A, *B;
  float* C;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 4 * 2));  // x2: GEMM_PROBE_EPI_FRESH
  __bf16* pre = nullptr;
  float* bias = nullptr;
  if (epi) {
    CK(hipMalloc(&pre, (size_t)M * N * 2 * 2));
    CK(hipMalloc(&bias, (size_t)N * 4));
    CK(hipMemset(bias, 0, (size_t)N * 4));
  }
  fill_kernel<<<1024, 256>>>(A, (size_t)M * K, 1u);
  fill_kernel<<<1024, 256>>>(B, (size_t)N * K, 2u);
  // mode 0: A [M][K], B [N][K]; 1: B [K][N]; 2: A [K][M], B [K][N] (accumulating, split-K)
  const int lda = mode == 2 ? M : K, ldb = mode == 0 ? K : N;
  const int flags = mode == 2 ? 8 : (epi ? 1 | 2 : 0);
  auto run = [&] {
    const int rc = mta_gemm_bf16(mode, A, B, M, N, K, lda, ldb, 1.f, flags, bias, nullptr, nullptr, nullptr, 0.f,
                                 nullptr, C, pre, N, N, ksplit, nullptr, 0, 0);
    if (rc) {
      printf("gemm rc=%d\n", rc);
      exit(1);
    }
  };
  for (int i = 0; i < 3; ++i) run();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < 20; ++r) {
    CK(hipEventRecord(e0, 0));
    run();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms * 1e3f);
  }
  std::sort(ts.begin(), ts.end());
  const double us = ts[ts.size() / 2];
  printf("gemm_probe M=%d N=%d K=%d mode=%d epi=%d: %.2f us  %.1f TFLOP/s\n", M, N, K, mode, epi, us,
         2.0 * M * N * K / (us * 1e-6) / 1e12);
#ifdef MTA_STAMPS
  unsigned long long zero[8][8] = {};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(big::stamp_acc), zero, sizeof(zero)));
  run();
  CK(hipDeviceSynchronize());
  unsigned long long acc[8][8];
  CK(hipMemcpyFromSymbol(acc, HIP_SYMBOL(big::stamp_acc), sizeof(acc)));
  const int tile = 256;
  const int blocks = ((M + tile - 1) / tile) * ((N + tile - 1) / tile) * ksplit;
  const int nk = K / 32 / ksplit;
  const char* names[8] = {"reads", "dma_wait_r1", "barrier1", "mfma_seg", "dma_wait_r0", "barrier2", "loop", "epilogue"};
  printf("cycles per k-tile (loop, epilogue: per tile) averaged over %d blocks, %d k-tiles\n", blocks, nk);
  printf("%-12s", "wave");
  for (int w = 0; w < 8; ++w) printf(" %7d", w);
  printf("\n");
  for (int i = 0; i < 8; ++i) {
    printf("%-12s", names[i]);
    for (int w = 0; w < 8; ++w)
      printf(" %7.0f", (double)acc[w][i] / blocks / (i == 7 ? 1 : (i == 6 ? 1 : nk)) / (i == 6 ? nk : 1));
    printf("\n");
  }
#ifdef GEMM_PROBE_EPI_TWICE
  unsigned long long e2[8];
  CK(hipMemcpyFromSymbol(e2, HIP_SYMBOL(big::epi2_acc), sizeof(e2)));
  printf("%-12s", "epilogue2");  // accumulated over the 24 timed + warm-up runs: per tile and run
  for (int w = 0; w < 8; ++w) printf(" %7.0f", (double)e2[w] / blocks / 24.0);
  printf("\n");
#endif
#endif
  return 0;
}
