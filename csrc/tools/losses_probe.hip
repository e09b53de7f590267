// Diagnostic probe (not part of the extension): times the one-launch training decoder of losses.hip at the
// headline shape (N=100 sequences, n=30 target days, H=64) and, in a -DMTA_STAMPS=1 build, prints the
// s_memtime cycles of its phases (staging, heads, losses, d(alpha,beta), dh + head grads).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc [-DMTA_STAMPS=1] csrc/tools/losses_probe.hip \
//         -o tools_bin/losses_probe
#include <cstdio>
#include <vector>

#include "../losses.hip"

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);       \
      return 1;                                                             \
    }                                                                       \
  } while (0)

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 100, n = 30, C = 4, H = 64;
  const int want_nll = argc > 2 ? atoi(argv[2]) : 0;
  std::vector<float> hy((size_t)N * n * C), hh((size_t)N * H), hw(H), hip(N, 1.5f), hf = {0.001f, 0.0002f};
  for (size_t i = 0; i < hy.size(); ++i) hy[i] = 0.01f * (float)((long)((i * 7919) % 101) - 50) / 50.f;
  for (size_t i = 0; i < hh.size(); ++i) hh[i] = (float)((long)((i * 104729) % 201) - 100) / 100.f;
  for (int i = 0; i < H; ++i) hw[i] = 0.1f * (float)((i * 31) % 17 - 8) / 8.f;
  float *y, *h, *wa, *wb, *ba, *bb, *fac, *ip, *out, *dh, *g;
  double* acc;
  CK(hipMalloc(&y, hy.size() * 4));
  CK(hipMalloc(&h, hh.size() * 4));
  CK(hipMalloc(&wa, H * 4));
  CK(hipMalloc(&wb, H * 4));
  CK(hipMalloc(&ba, 4));
  CK(hipMalloc(&bb, 4));
  CK(hipMalloc(&fac, 8));
  CK(hipMalloc(&ip, N * 4));
  CK(hipMalloc(&out, 16));
  CK(hipMalloc(&dh, (size_t)N * H * 4));
  CK(hipMalloc(&g, (2 * H + 2) * 4));
  CK(hipMalloc(&acc, 64));
  CK(hipMemcpy(y, hy.data(), hy.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(h, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(wa, hw.data(), H * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(wb, hw.data(), H * 4, hipMemcpyHostToDevice));
  CK(hipMemset(ba, 0, 4));
  CK(hipMemset(bb, 0, 4));
  CK(hipMemcpy(fac, hf.data(), 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(ip, hip.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemset(g, 0, (2 * H + 2) * 4));
  CK(hipMemset(acc, 0, 64));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  double ms = 0;
  const int reps = 200;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a));
    mta_heads_losses_train(h, H, wa, ba, wb, bb, y, fac, ip, N, n, C, 1, N, 0, want_nll, 1.f, 1.f, 1.f, out, acc, dh,
                           g, g + H, g + H + 1, g + 2 * H + 1, N, 0);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float m;
    CK(hipEventElapsedTime(&m, a, b));
    if (r >= 20) ms += m / (reps - 20);
  }
  printf("N=%d want_nll=%d: heads_losses_train %.2f us/launch\n", N, want_nll, ms * 1e3);
  // one fresh call for the values (the head gradients accumulate)
  CK(hipMemset(g, 0, (2 * H + 2) * 4));
  mta_heads_losses_train(h, H, wa, ba, wb, bb, y, fac, ip, N, n, C, 1, N, 0, want_nll, 1.f, 1.f, 1.f, out, acc, dh,
                         g, g + H, g + H + 1, g + 2 * H + 1, N, 0);
  CK(hipDeviceSynchronize());
  std::vector<float> ho(4), hdh((size_t)N * H), hg(2 * H + 2);
  CK(hipMemcpy(ho.data(), out, 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hdh.data(), dh, hdh.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hg.data(), g, hg.size() * 4, hipMemcpyDeviceToHost));
  double sdh = 0, sg = 0;
  for (size_t i = 0; i < hdh.size(); ++i) sdh += hdh[i] * (1.0 + i % 7);
  for (size_t i = 0; i < hg.size(); ++i) sg += hg[i] * (1.0 + i % 5);
  printf("  out = %.9g %.9g %.9g %.9g  dh.w = %.9g  g.w = %.9g  g_ba = %.9g g_bb = %.9g\n", ho[0], ho[1], ho[2],
         ho[3], sdh, sg, hg[H], hg[2 * H + 1]);
#if MTA_STAMPS
  unsigned long long st[8];
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(mta_loss_stamps), sizeof(st)));
  const char* nm[5] = {"stage y,h", "heads", "losses", "d(alpha,beta)", "dh+head grads"};
  for (int k = 0; k < 5; ++k) printf("  %-14s %6llu cycles\n", nm[k], st[k + 1] - st[k]);
#endif
  return 0;
}
