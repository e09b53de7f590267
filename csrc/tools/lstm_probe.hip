// Diagnostic probe (not part of the extension): runs the LSTM recurrence kernels alone on
// random data and prints per-segment cycle shares from in-kernel s_memtime stamps.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc -DMTA_STAMPS=1 csrc/tools/lstm_probe.hip -o build/lstm_probe
// Stamp builds are slower than the real kernel: read the SHARES, not the absolute length.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../lstm.hip"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static float* dev_rand(size_t n, float scale) {
  std::vector<float> h(n);
  for (auto& v : h) v = scale * (2.f * rand() / RAND_MAX - 1.f);
  float* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int H = 64, T = 60, N = argc > 1 ? atoi(argv[1]) : 100, Np = (N + 15) / 16 * 16;
  const int prec = argc > 2 ? atoi(argv[2]) : PREC_BF16X3;
  float* x = dev_rand((size_t)N * T * 3, 1.f);
  float* wih = dev_rand(4 * H * 3, 0.125f);
  float* bih = dev_rand(4 * H, 0.125f);
  float* bhh = dev_rand(4 * H, 0.125f);
  float* whh = dev_rand(4 * H * H, 0.125f);
  float* gx = dev_rand((size_t)T * Np * 4 * H, 1.f);
  float *stash, *hseq, *dG, *dhl;
  CK(hipMalloc(&stash, (size_t)T * Np * 5 * H * 4));
  CK(hipMalloc(&hseq, (size_t)T * Np * H * 4));
  CK(hipMalloc(&dG, (size_t)T * Np * 4 * H * 4));
  dhl = dev_rand((size_t)N * H, 1.f);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[3] = {"fwd fused-x (FIN=3)", "fwd gx (FIN=0)", "bwd"};
  for (int which = 0; which < 3; ++which) {
    float ms = 0;
    for (int rep = 0; rep < 20; ++rep) {
      CK(hipEventRecord(a));
      if (which == 0) mta_lstm_fwd_layer(H, prec, x, wih, bih, bhh, 3, nullptr, stash, whh, hseq, N, Np, T, 0);
      else if (which == 1) mta_lstm_fwd_layer(H, prec, nullptr, nullptr, nullptr, nullptr, 0, gx, stash, whh, hseq, N, Np, T, 0);
      else mta_lstm_bwd_layer(H, prec, stash, whh, nullptr, dhl, dG, N, Np, T, 0);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float m;
      CK(hipEventElapsedTime(&m, a, b));
      if (rep >= 5) ms += m / 15;
    }
    unsigned long long acc[2][8];
    CK(hipMemcpyFromSymbol(acc, HIP_SYMBOL(mta_stamp_acc), sizeof(acc)));
    const int k = which == 2 ? 1 : 0;
    unsigned long long tot = 0;
    for (int s = 1; s < 8; ++s) tot += acc[k][s];
    printf("%-22s N=%d prec=%d  %.1f us/launch (%.2f us/step)  cycles/step:", names[which], N, prec, ms * 1e3,
           ms * 1e3 / T);
    for (int s = 1; s < 6; ++s) printf(" seg%d=%.0f", s, (double)acc[k][s] / T);
    printf("  total=%.0f\n", (double)tot / T);
  }
  return 0;
}
