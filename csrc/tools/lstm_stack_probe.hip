// Diagnostic probe (not part of the extension): times the layer-pipelined LSTM kernels of lstm_stack.hip
// (forward, and backward with the fused weight gradients) on random data at the headline shape, and in a
// -DMTA_STAMPS=1 build prints per-segment s_memtime cycles per step of block 0 for each wave role.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc [-DMTA_STAMPS=1|2] \
//         csrc/tools/lstm_stack_probe.hip -o tools_bin/lstm_stack_probe
//   ./tools_bin/lstm_stack_probe [N=100] [L=2] [prec=1] [T=60]
// Stamp builds are slower than the real kernel (each stamp waits lgkmcnt): read the SHARES there and the
// absolute times from the stamp-free build.
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "../lstm_stack.hip"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);            \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

static float* dev_rand(size_t n, float scale) {
  std::vector<float> h(n);
  for (auto& v : h) v = scale * (2.f * rand() / RAND_MAX - 1.f);
  float* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}
static float* dev_zero(size_t n) {
  float* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemset(d, 0, n * 4));
  return d;
}

int main(int argc, char** argv) {
  const int H = 64, FIN = 3;
  const int N = argc > 1 ? atoi(argv[1]) : 100;
  const int L = argc > 2 ? atoi(argv[2]) : 2;
  const int prec = argc > 3 ? atoi(argv[3]) : PREC_BF16X3;
  const int T = argc > 4 ? atoi(argv[4]) : 60;
  // mode 0: training with dropout 0.2 (the headline step); 1: training, no dropout; 2: inference (no stash)
  const int mode = argc > 5 ? atoi(argv[5]) : 0;
  const float p = mode == 0 ? 0.2f : 0.0f;
  const int Np = (N + 15) / 16 * 16;
  if (L < 1 || L > 8 || N < 1 || T < 4 || T > 1000) {
    printf("bad arguments\n");
    return 1;
  }
  const float k = 0.125f;
  float* x = dev_rand((size_t)N * T * FIN, 1.f);
  std::vector<float*> wih(L), whh(L), bih(L), bhh(L), hseq(L), xdrop(L, nullptr), stash(L), dG(L), dX(L, nullptr),
      inp(L), gwih(L), gwhh(L), gbih(L), gbhh(L);
  std::vector<uint32_t*> mask(L, nullptr);
  for (int l = 0; l < L; ++l) {
    const int fin = l == 0 ? FIN : H;
    wih[l] = dev_rand((size_t)4 * H * fin, k);
    whh[l] = dev_rand((size_t)4 * H * H, k);
    bih[l] = dev_rand(4 * H, k);
    bhh[l] = dev_rand(4 * H, k);
    hseq[l] = dev_zero((size_t)T * Np * H);
    if (l >= 1 && mode == 0) {
      xdrop[l] = dev_zero((size_t)T * Np * H);
      CK(hipMalloc(&mask[l], (size_t)T * Np * H));
    }
    if (l < L - 1) dX[l] = dev_zero((size_t)2 * T * Np * H);  // room for the granule hand-off (8 bytes per value)
    stash[l] = mode == 2 ? nullptr : dev_zero((size_t)T * Np * 5 * H);
    dG[l] = dev_zero((size_t)T * Np * 4 * H);
    gwih[l] = dev_zero((size_t)4 * H * fin);
    gwhh[l] = dev_zero((size_t)4 * H * H);
    gbih[l] = dev_zero(4 * H);
    gbhh[l] = dev_zero(4 * H);
    inp[l] = l == 0 ? x : (mode == 0 ? xdrop[l] : hseq[l - 1]);
  }
  float* dh_last = dev_rand((size_t)N * H, 1.f);
  uint64_t* seeds;
  CK(hipMalloc(&seeds, 8 * sizeof(uint64_t)));
  std::vector<uint64_t> hs(8);
  for (int i = 0; i < 8; ++i) hs[i] = 0x1234567ull * (i + 1);
  CK(hipMemcpy(seeds, hs.data(), 8 * sizeof(uint64_t), hipMemcpyHostToDevice));
  // decoupled forward (default; DEC=0 in the environment selects the barrier form): (L - 1) x (T, Np, H) granules
  const int dec = getenv("DEC") && atoi(getenv("DEC")) == 0 ? 0 : 1;
  const int bform = 0;  // backward dX hand-off: fp32 rows + progress words
  const int bgran = bform == 1;
  const int nowg = getenv("NOWG") && atoi(getenv("NOWG")) == 1;  // 1: no fused weight-gradient workgroups (A/B)
  unsigned long long* gran = nullptr;
  CK(hipMalloc(&gran, (size_t)(L > 1 ? L - 1 : 1) * T * Np * H * 8));
  CK(hipMemset(gran, 0, (size_t)(L > 1 ? L - 1 : 1) * T * Np * H * 8));
  unsigned* flags;
  const long nflags = mta_lstm_stack_flag_words(Np);
  CK(hipMalloc(&flags, nflags * 4));
  CK(hipMemset(flags, 0, nflags * 4));

#if STACK_STAMPS
  // stamp the last layer's first tile in the forward (its input waves run the W_ih MFMAs: the slowest layer)
  // and the top layer's first tile in the backward (block 0: its gradient waves run the dx MFMAs)
  const int ntiles = Np / 16, tr8 = (ntiles + 7) / 8 * 8;
  const int which = argc > 6 ? atoi(argv[6]) : L - 1;
  // BWDL=<layer> stamps that layer's first tile in the backward (default: the top layer)
  const int bl = getenv("BWDL") ? atoi(getenv("BWDL")) : L - 1;
  int sb[2] = {which * tr8, (L - 1 - bl) * tr8};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(mta_stack_stamp_block), sb, sizeof(sb)));
  printf("stamping forward layer %d (block %d), backward layer %d (block %d)\n", which, sb[0], bl, sb[1]);
#endif
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 200, skip = 20;
  double ms_f = 0, ms_b = 0;
  for (int rep = 0; rep < reps; ++rep) {
    float m;
    CK(hipEventRecord(a));
    int rc = mta_lstm_stack_fwd(H, prec, L, FIN, x, wih.data(), whh.data(), bih.data(), bhh.data(), hseq.data(),
                                xdrop.data(), mask.data(), stash.data(), seeds, p, flags, N, Np, T, gran, dec, 0);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    if (rc) {
      printf("fwd rc=%d\n", rc);
      return 1;
    }
    CK(hipEventElapsedTime(&m, a, b));
    if (rep >= skip) ms_f += m / (reps - skip);
    if (mode == 2) continue;
    CK(hipEventRecord(a));
    rc = mta_lstm_stack_bwd(H, prec, L, FIN, stash.data(), whh.data(), wih.data(), dh_last, dG.data(), dX.data(),
                            hseq.data(), inp.data(), gwih.data(), nowg ? nullptr : gwhh.data(), gbih.data(), gbhh.data(),
                            const_cast<const uint32_t* const*>(mask.data()), nullptr, seeds, p,
                            mode == 0 ? 1 : 0, flags, N, Np, T, bform, 0);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    if (rc) {
      printf("bwd rc=%d\n", rc);
      return 1;
    }
    CK(hipEventElapsedTime(&m, a, b));
    if (rep >= skip) ms_b += m / (reps - skip);
  }
#if STACK_TIMELINE
  {
    constexpr int MAXL_PROBE = 8;
    // the last forward / backward of the timed loop, per layer: entry / loop start / step T/2 / end, in ns (100 MHz
    // real-time counter) from the earliest entry of the same tile over its layers, averaged over tiles
    unsigned long long tl[2][64][4];
    CK(hipMemcpyFromSymbol(tl, HIP_SYMBOL(mta_stack_tl), sizeof(tl)));
    const int ntl = Np / 16, tr8l = (ntl + 7) / 8 * 8;
    for (int d = 0; d < 2; ++d) {
      auto blk = [&](int l, int i) { return (d == 0 ? l : L - 1 - l) * tr8l + i; };
      double v[MAXL_PROBE][4] = {};
      int cnt[MAXL_PROBE] = {};
      for (int i = 0; i < ntl; ++i) {
        unsigned long long t0 = ~0ull;
        bool ok = true;
        for (int l = 0; l < L; ++l) {
          if (blk(l, i) >= 64) { ok = false; break; }
          t0 = tl[d][blk(l, i)][0] < t0 ? tl[d][blk(l, i)][0] : t0;
        }
        if (!ok) continue;
        for (int l = 0; l < L; ++l) {
          ++cnt[l];
          for (int k = 0; k < 4; ++k) v[l][k] += (double)(long long)(tl[d][blk(l, i)][k] - t0);
        }
      }
      for (int l0 = 0; l0 < L; ++l0) {
        const int l = d == 0 ? l0 : L - 1 - l0;
        if (!cnt[l]) continue;
        const double n = cnt[l];
        const int half = d == 0 ? T - 1 - T / 2 : T / 2;
        printf("timeline %s layer %d (ns from the tile's first entry, mean of %d tiles): entry %.0f start %.0f mid "
               "%.0f end %.0f  -> pace %.0f ns/step (second half)\n",
               d == 0 ? "fwd" : "bwd", l, cnt[l], 10 * v[l][0] / n, 10 * v[l][1] / n, 10 * v[l][2] / n,
               10 * v[l][3] / n, 10 * (v[l][3] - v[l][2]) / n / half);
      }
    }
    {
      // the backward's last weight-gradient workgroups (the bottom layer's earliest chunks), ns from the first
      // recurrence entry of the launch (one real-time clock for the whole chip)
      unsigned long long tw[64][4];
      CK(hipMemcpyFromSymbol(tw, HIP_SYMBOL(mta_stack_tlw), sizeof(tw)));
      unsigned long long r0 = ~0ull, rend = 0;
      for (int b = 0; b < L * tr8l && b < 64; ++b)
        if (b % tr8l < ntl) {
          r0 = tl[1][b][0] < r0 ? tl[1][b][0] : r0;
          rend = tl[1][b][3] > rend ? tl[1][b][3] : rend;
        }
      if (!nowg) {
        unsigned long long ts[18];
        CK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(mta_stack_tls), sizeof(ts)));
        printf("wgrad last block slices (ns from ready):");
        for (int k = 0; k < 18; ++k)
          if (ts[k] >= tw[0][1] && ts[k] - tw[0][1] < 10000000ull) printf(" [%d]%.0f", k, 10.0 * (double)(ts[k] - tw[0][1]));
        printf("\n");
        printf("wgrad tail: recurrence (%d blocks <64) ends at %.0f ns\n", L * tr8l, 10.0 * (double)(rend - r0));
        for (int r = 0; r < 12; ++r)
          printf("  wgrad block last-%d: entry %.0f ready %.0f body_done %.0f exit %.0f ns\n", r,
                 10.0 * (double)(long long)(tw[r][0] - r0), 10.0 * (double)(long long)(tw[r][1] - r0),
                 10.0 * (double)(long long)(tw[r][2] - r0), 10.0 * (double)(long long)(tw[r][3] - r0));
      }
    }
  }
#endif
  // determinism: two forwards with the same seeds must agree bitwise (h of every layer at every step)
  {
    std::vector<std::vector<float>> ref(L), again(L);
    for (int pass = 0; pass < 2; ++pass) {
      CK(hipMemcpy(seeds, hs.data(), 8 * sizeof(uint64_t), hipMemcpyHostToDevice));
      int rc = mta_lstm_stack_fwd(H, prec, L, FIN, x, wih.data(), whh.data(), bih.data(), bhh.data(), hseq.data(),
                                  xdrop.data(), mask.data(), stash.data(), seeds, p, flags, N, Np, T, gran, dec, 0);
      CK(hipDeviceSynchronize());
      if (rc) return 1;
      for (int l = 0; l < L; ++l) {
        auto& v = pass ? again[l] : ref[l];
        v.resize((size_t)T * Np * H);
        CK(hipMemcpy(v.data(), hseq[l], v.size() * 4, hipMemcpyDeviceToHost));
      }
    }
    long bad = 0;
    double maxd = 0;
    for (int l = 0; l < L; ++l)
      for (int t = 0; t < T; ++t)
        for (int n = 0; n < N; ++n)
          for (int u = 0; u < H; ++u) {
            const size_t i = ((size_t)t * Np + n) * H + u;
            const double d = fabs((double)ref[l][i] - again[l][i]);
            if (d != 0) ++bad;
            if (d > maxd) maxd = d;
          }
    printf("determinism: %ld of %ld h values differ between two identical forwards (max |d| %.3e)\n", bad,
           (long)L * T * N * H, maxd);
  }
  // backward determinism: 6 backwards of the same forward state must give bitwise-identical dG (the fused weight
  // gradients' atomics aside); per layer, the first differing step (reverse order) of each rerun
  if (mode != 2) {
    std::vector<std::vector<float>> ref(L), again(L);
    int nbad = 0;
    for (int pass = 0; pass < 6; ++pass) {
      CK(hipMemcpy(seeds, hs.data(), 8 * sizeof(uint64_t), hipMemcpyHostToDevice));
      int rc = mta_lstm_stack_bwd(H, prec, L, FIN, stash.data(), whh.data(), wih.data(), dh_last, dG.data(), dX.data(),
                                  hseq.data(), inp.data(), gwih.data(), nowg ? nullptr : gwhh.data(), gbih.data(),
                                  gbhh.data(), const_cast<const uint32_t* const*>(mask.data()), nullptr, seeds, p,
                                  mode == 0 ? 1 : 0, flags, N, Np, T, bform, 0);
      CK(hipDeviceSynchronize());
      if (rc) return 1;
      char line[512];
      int off = 0;
      bool any = false;
      for (int l = 0; l < L; ++l) {
        auto& v = pass ? again[l] : ref[l];
        v.resize((size_t)T * Np * 4 * H);
        CK(hipMemcpy(v.data(), dG[l], v.size() * 4, hipMemcpyDeviceToHost));
        if (!pass) continue;
        int first = -1;
        for (int t = T - 1; t >= 0 && first < 0; --t)
          for (int n = 0; n < N && first < 0; ++n)
            for (int c = 0; c < 4 * H; ++c) {
              const size_t i = ((size_t)t * Np + n) * 4 * H + c;
              if (ref[l][i] != again[l][i]) { first = t; break; }
            }
        if (first >= 0) any = true;
        off += snprintf(line + off, sizeof(line) - off, " L%d:%d", l, first);
      }
      if (pass) {
        nbad += any;
        if (any) printf("bwd determinism: rerun %d differs (first differing step per layer, -1 = none):%s\n", pass, line);
      }
    }
    printf("bwd determinism: %d of 5 reruns differ\n", nbad);
  }
  // checksums (variants of the kernel must agree): last layer's h at T-1 and layer 0's W_hh gradient after reps runs
  {
    std::vector<float> hl((size_t)Np * H), gw((size_t)4 * H * H);
    CK(hipMemcpy(hl.data(), hseq[L - 1] + (size_t)(T - 1) * Np * H, hl.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gw.data(), gwhh[0], gw.size() * 4, hipMemcpyDeviceToHost));
    double s1 = 0, s2 = 0;
    for (int n = 0; n < N; ++n)
      for (int u = 0; u < H; ++u) s1 += (double)hl[(size_t)n * H + u] * (1 + (n * 7 + u) % 5);
    for (size_t i = 0; i < gw.size(); ++i) s2 += (double)gw[i] * (1 + i % 3);
    printf("checksum h=%.9e gwhh=%.9e\n", s1, s2);
  }
  unsigned tmo = 0;
  CK(hipMemcpy(&tmo, flags + (nflags - 160), 4, hipMemcpyDeviceToHost));
  printf("dec=%d bform=%d mode=%d N=%d L=%d T=%d prec=%d stamps=%d: fwd %.1f us (%.3f us/step)  bwd %.1f us (%.3f us/step)  "
         "timeouts=%u\n",
         dec, bform, mode, N, L, T, prec, MTA_STAMPS, ms_f * 1e3, ms_f * 1e3 / T, ms_b * 1e3, ms_b * 1e3 / T,
         tmo);
#if STACK_STAMPS
  unsigned long long acc[2][3][8];
  CK(hipMemcpyFromSymbol(acc, HIP_SYMBOL(mta_stack_stamp_acc), sizeof(acc)));
  const char* seg[2][3][8] = {
      {{"", "gx_lds_read", "mfma_chain", "activations", "lds_write", "barrier", "", ""},
       {"", "vmcnt_drain+flag", "store_step", "barrier", "", "", "", ""},
       {"", "write_x(load_wait)", "compute_gx", "poll+load_issue", "barrier", "", "", ""}},
      {{"", "dh_lds_read", "vmcnt_wait", "dG_store_issue", "elementwise+lds", "stash_prefetch", "barrier",
        "mfma_dh"},
       {"", "vmem_wait", "flags+stage+loads", "dx_step", "barrier", "", "", ""},
       {"", "", "", "", "", "", "", ""}}};
  if (dec) {  // the decoupled forward's segments (csrc/lstm_stack.hip stack_fwd_dec)
    const char* d0[3][8] = {{"", "gx_wait+read", "h_wait", "a_read+stage+mfma", "activations", "h_write+post", "", ""},
                            {"", "stg_wait", "lds_read+post", "stores", "", "", "", ""},
                            {"", "slot/xq_wait", "gx_compute+post", "x_ready(poll)", "x_write+issue", "", "", ""}};
    for (int r = 0; r < 3; ++r)
      for (int k = 0; k < 8; ++k) seg[0][r][k] = d0[r][k];
  }
  const char* dir[2] = {"fwd", "bwd"};
  const char* role[2][3] = {{"recurrent", "store", "input"}, {"recurrent", "gradient", ""}};
  for (int d = 0; d < 2; ++d)
    for (int r = 0; r < 3; ++r) {
      if (!role[d][r][0]) continue;
      unsigned long long tot = 0;
      for (int s = 1; s < 8; ++s) tot += acc[d][r][s];
      printf("  %s %-9s cycles/step total=%6.0f :", dir[d], role[d][r], (double)tot / T);
      for (int s = 1; s < 8; ++s)
        if (seg[d][r][s][0]) printf(" %s=%.0f", seg[d][r][s], (double)acc[d][r][s] / T);
      printf("\n");
    }
#endif
  return tmo ? 3 : 0;  // a hand-off that gave up waiting: the results are invalid
}
