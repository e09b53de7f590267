// Sanitizer driver for the host prefetcher (csrc/host/prefetch.cpp), built and run WITHOUT the GPU:
//   python -m masters_thesis_amd.ops.build --sanitize      (AddressSanitizer+UBSan and ThreadSanitizer builds)
// Exercises the ring protocol from a consumer thread while worker threads fill slots: several epochs, every
// batch checked row by row, releases out of lock-step with fills, early stops while workers are mid-fill,
// restart on the same object and destroy with workers running.  Exits non-zero on any mismatch; the
// sanitizers abort on memory errors, undefined behaviour and data races.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

extern "C" {
void* mta_prefetch_create(int ntensors, const void* const* host, const long* row_bytes, void* const* staging, int B,
                          int R, int nthreads);
void mta_prefetch_start(void* h, const long* idx, long n_idx, long n_batches);
int mta_prefetch_wait(void* h, long batch, long timeout_ms);
int mta_prefetch_ready(void* h, long batch);
void mta_prefetch_release(void* h, long batch);
void mta_prefetch_stop(void* h);
void mta_prefetch_destroy(void* h);
}

static int check(bool ok, const char* what, long b) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s (batch %ld)\n", what, b);
    std::exit(1);
  }
  return 0;
}

int main() {
  std::mt19937 rng(1234);
  const int rows = 97;
  const long rb0 = 7 * 3 * sizeof(float), rb1 = 2 * sizeof(float);
  std::vector<float> X(rows * 21), F(rows * 2);
  for (size_t i = 0; i < X.size(); ++i) X[i] = (float)i;
  for (size_t i = 0; i < F.size(); ++i) F[i] = -(float)i;
  const int configs[][3] = {{1, 2, 1}, {3, 4, 2}, {4, 3, 4}, {8, 2, 3}};
  for (const auto& c : configs) {
    const int B = c[0], R = c[1], T = c[2];
    std::vector<char> s0(R * B * rb0), s1(R * B * rb1);
    const void* host[2] = {X.data(), F.data()};
    const long rbytes[2] = {rb0, rb1};
    void* staging[2] = {s0.data(), s1.data()};
    void* h = mta_prefetch_create(2, host, rbytes, staging, B, R, T);
    check(h != nullptr, "create", -1);
    for (int epoch = 0; epoch < 6; ++epoch) {
      std::vector<long> idx(rows);
      std::iota(idx.begin(), idx.end(), 0L);
      std::shuffle(idx.begin(), idx.end(), rng);
      const long nb = rows / B;
      mta_prefetch_start(h, idx.data(), (long)idx.size(), nb);
      // odd epochs stop early, while workers may be filling
      const long upto = (epoch & 1) ? nb / 2 : nb;
      for (long b = 0; b < upto; ++b) {
        const int slot = mta_prefetch_wait(h, b, 10000);
        check(slot == (int)(b % R), "wait slot", b);
        for (int j = 0; j < B; ++j) {
          const long r = idx[b * B + j];
          check(std::memcmp(s0.data() + (slot * B + j) * rb0, (const char*)X.data() + r * rb0, rb0) == 0, "X row", b);
          check(std::memcmp(s1.data() + (slot * B + j) * rb1, (const char*)F.data() + r * rb1, rb1) == 0, "F row", b);
        }
        if (b + R < nb) check(!mta_prefetch_ready(h, b + R), "slot refilled before release", b);
        mta_prefetch_release(h, b);
      }
      if (epoch == 3) mta_prefetch_stop(h);
    }
    mta_prefetch_destroy(h);  // workers of the last (early-stopped) epoch still running
  }
  std::printf("prefetch_stress: OK\n");
  return 0;
}
