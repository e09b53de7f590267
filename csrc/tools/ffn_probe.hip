// Diagnostic probe (not part of the extension): the fused transformer FFN half (csrc/tr_ffn.hip) forward and backward
// on the transformer_encoder B=1 shape (M = 104 x 60 tokens), timed with events, and (built with -DMTA_STAMPS=1)
// the s_memtime split of every workgroup's critical path: phase means over the workgroups, plus the spread of their
// start and end times (how long the launch takes to fill and drain).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc [-DMTA_STAMPS=1] \
//         csrc/tools/ffn_probe.hip -o tools_bin/ffn_probe[_s]
//   ./tools_bin/ffn_probe [M] [nn]      (nn = 1: the transposed weight-gradient operand outputs, the default path)
#include "../tr_ffn.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);           \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void fill_bf16(__bf16* p, size_t n, uint32_t seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 0x9E3779B1u ^ seed;
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    p[i] = (__bf16)(scale * ((float)(x & 0xFFFF) / 32768.f - 1.f));
  }
}
__global__ void fill_f32(float* p, size_t n, uint32_t seed, float scale, float bias) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 0x9E3779B1u ^ seed;
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    p[i] = bias + scale * ((float)(x & 0xFFFF) / 32768.f - 1.f);
  }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 104 * 60;
  const int nn = argc > 2 ? atoi(argv[2]) : 1;
  const size_t md = (size_t)M * FD, mf = (size_t)M * FF;
  __bf16 *w1, *w2, *w1t, *w2t, *xn2, *pre, *u, *uT, *xn2T, *dxb, *dpre, *dx1b, *dpreT, *dxT;
  float *b1, *b2, *g2, *x1, *r2, *x2, *dx, *dx1, *dg2;
  CK(hipMalloc(&w1, FF * FD * 2));
  CK(hipMalloc(&w2, FF * FD * 2));
  CK(hipMalloc(&w1t, FF * FD * 2));
  CK(hipMalloc(&w2t, FF * FD * 2));
  CK(hipMalloc(&b1, FF * 4));
  CK(hipMalloc(&b2, FD * 4));
  CK(hipMalloc(&g2, FD * 4));
  CK(hipMalloc(&dg2, FD * 4));
  for (__bf16** p : {&xn2, &dxb, &dx1b, &xn2T, &dxT}) CK(hipMalloc(p, md * 2));
  for (__bf16** p : {&pre, &u, &uT, &dpre, &dpreT}) CK(hipMalloc(p, mf * 2));
  for (float** p : {&x1, &x2, &dx, &dx1}) CK(hipMalloc(p, md * 4));
  CK(hipMalloc(&r2, (size_t)M * 4));
  fill_bf16<<<256, 256>>>(w1, FF * FD, 1u, 0.09f);
  fill_bf16<<<256, 256>>>(w2, FF * FD, 2u, 0.05f);
  fill_bf16<<<256, 256>>>(w1t, FF * FD, 3u, 0.09f);
  fill_bf16<<<256, 256>>>(w2t, FF * FD, 4u, 0.05f);
  fill_f32<<<256, 256>>>(b1, FF, 5u, 0.1f, 0.f);
  fill_f32<<<256, 256>>>(b2, FD, 6u, 0.1f, 0.f);
  fill_f32<<<256, 256>>>(g2, FD, 7u, 0.1f, 1.f);
  fill_f32<<<1024, 256>>>(x1, md, 8u, 1.f, 0.f);
  fill_f32<<<1024, 256>>>(dx, md, 9u, 1e-3f, 0.f);
  fill_bf16<<<1024, 256>>>(dxb, md, 10u, 1e-3f);
  CK(hipDeviceSynchronize());
  auto fwd = [&] {
    const int rc = mta_tr_ffn(0, M, FD, FF, 1e-6f, w1, w2, b1, b2, g2, x1, nullptr, 0.f, nn ? nullptr : xn2, pre,
                              nn ? nullptr : u, r2, x2, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                              nullptr, nn ? uT : nullptr, nn ? xn2T : nullptr, nullptr, nullptr, 0);
    if (rc) {
      printf("fwd rc=%d\n", rc);
      exit(1);
    }
  };
  auto bwd = [&] {
    const int rc = mta_tr_ffn(1, M, FD, FF, 0.f, w1t, w2t, nullptr, nullptr, g2, x1, nullptr, 0.f, nullptr, nullptr,
                              nullptr, nullptr, nullptr, dxb, dx, r2, pre, nn ? nullptr : dpre, dx1, dx1b, dg2, nullptr,
                              nullptr, nn ? dpreT : nullptr, nn ? dxT : nullptr, 0);
    if (rc) {
      printf("bwd rc=%d\n", rc);
      exit(1);
    }
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int dir = 0; dir < 2; ++dir) {
    auto run = [&] { dir == 0 ? fwd() : bwd(); };
    for (int i = 0; i < 20; ++i) run();
    CK(hipDeviceSynchronize());
    // spaced single launches (each waits for the previous): the per-launch latency the graphed step sees
    float tot = 0.f;
    const int reps = 50;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0, 0));
      run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tot += ms;
    }
    printf("%s M=%d nn=%d grid=%d: %.2f us per launch (event-bracketed, %d reps)\n", dir ? "bwd" : "fwd", M, nn,
           (M + FBM - 1) / FBM, 1e3f * tot / reps, reps);
#if MTA_STAMPS
    run();
    CK(hipDeviceSynchronize());
    static unsigned long long st[2][256][12];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(mta_ffn_stamp), sizeof(st)));
    const int nb = std::min(256, (M + FBM - 1) / FBM), np = dir ? 8 : 9;
    unsigned long long t0 = ~0ull, tend = 0, tlast_start = 0, tfirst_end = ~0ull;
    double ph[12] = {0}, lat = 0;
    for (int b = 0; b < nb; ++b) {
      t0 = std::min(t0, st[dir][b][10]);
      tlast_start = std::max(tlast_start, st[dir][b][10]);
      tend = std::max(tend, st[dir][b][11]);
      tfirst_end = std::min(tfirst_end, st[dir][b][11]);
      lat += (double)(st[dir][b][11] - st[dir][b][10]) / nb;
      for (int k = 1; k < np; ++k) ph[k] += (double)(st[dir][b][k] - st[dir][b][k - 1]) / nb;
    }
    printf("  100 MHz clock (10 ns): first start -> last start %llu, first start -> first end %llu, -> last end %llu, "
           "mean workgroup %.1f\n  mean phase split (shader cycles):", tlast_start - t0, tfirst_end - t0, tend - t0, lat);
    for (int k = 1; k < np; ++k) printf(" p%d=%.0f", k, ph[k]);
    printf("\n");
#endif
  }
  return 0;
}
