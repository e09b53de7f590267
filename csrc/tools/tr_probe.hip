// Diagnostic probe (not part of the extension): the fused transformer block forward (csrc/transformer.hip) at the
// transformer_encoder B=1 shape (100 sequences x 60 tokens, d 128), timed, and with -DMTA_TR_STAMPS the s_memtime
// split of its phases (summed over workgroups, wave 0).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc [-DMTA_TR_STAMPS] csrc/tools/tr_probe.hip -o tools_bin/tr_probe
#include "../transformer.hip"

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

template <class T>
T* dalloc(size_t n) {
  T* p;
  CK(hipMalloc(&p, n * sizeof(T)));
  CK(hipMemset(p, 0, n * sizeof(T)));
  return p;
}

int main(int argc, char** argv) {
  const int nseq = argc > 1 ? atoi(argv[1]) : 100, T = 60, M = nseq * T;
  std::vector<float> hx((size_t)M * 128);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
  float* xs = dalloc<float>(hx.size());
  CK(hipMemcpy(xs, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  auto w = [](size_t n) { return dalloc<__bf16>(n); };
  __bf16 *wqkv = w(384 * 128), *wo = w(128 * 128), *w1 = w(512 * 128), *w2 = w(128 * 512);
  float *g1 = dalloc<float>(128), *bqkv = dalloc<float>(384), *bo = dalloc<float>(128), *g2 = dalloc<float>(128);
  float *b1 = dalloc<float>(512), *b2 = dalloc<float>(128);
  __bf16 *xn = w((size_t)M * 128), *qkv = w((size_t)M * 384), *o = w((size_t)M * 128), *xn2 = w((size_t)M * 128);
  __bf16 *pre1 = w((size_t)M * 512), *u = w((size_t)M * 512);
  float *x1 = dalloc<float>((size_t)M * 128), *x2 = dalloc<float>((size_t)M * 128), *r1 = dalloc<float>(M);
  float *r2 = dalloc<float>(M), *lse = dalloc<float>((size_t)nseq * 4 * 64), *rope = dalloc<float>(T * 32);
  auto run = [&] {
    if (mta_tr_layer_fwd(nseq, T, 128, 512, 4, xs, wqkv, wo, w1, w2, g1, bqkv, bo, g2, b1, b2, 1e-6f, xn, qkv, o, xn2,
                         pre1, u, x1, x2, r1, r2, lse, rope, nullptr, 0.f, 0) != 0) {
      printf("launch failed\n");
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
  printf("tr_layer_fwd nseq=%d: %.2f us\n", nseq, ts[ts.size() / 2]);
#ifdef MTA_TR_STAMPS
  unsigned long long z[16] = {};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(tr_stamp), z, sizeof(z)));
  run();
  CK(hipDeviceSynchronize());
  unsigned long long acc[16];
  CK(hipMemcpyFromSymbol(acc, HIP_SYMBOL(tr_stamp), sizeof(acc)));
  const char* names[7] = {"loads(prm,x,seed)", "norm1+chunk0", "qkv(3 chunks)", "attention", "proj+norm2", "ffn",
                          "x2 store"};
  for (int i = 0; i < 7; ++i) printf("  %-20s %8.0f cycles per workgroup\n", names[i], (double)acc[i] / nseq);
#endif
  return 0;
}
