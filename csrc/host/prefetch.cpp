// Native host-side batch prefetcher for the streaming data path (residency=stream).
//
// Reference behaviour being replaced: torch DataLoader(num_workers=4, pin_memory=True)
// (`src/data.py:236-241`): worker processes collate a batch, a pin thread copies it to
// page-locked memory, and the training loop issues the H2D copy.  Here worker THREADS
// (no processes, no pickling) gather the rows of the next batches straight into a ring of
// R page-locked staging slots; the Python side issues one hipMemcpyAsync per tensor on a
// side HIP stream into the matching slot of a device ring, and the captured step graph
// gathers from that ring (csrc/lstm_aux.hip gather_batch_kernel).
//
// Protocol (all batch ids are per epoch, 0..n_batches-1, slot = batch % R):
//   worker w fills batches b = w, w+nthreads, ...   once b < released + R   (slot is free)
//   wait(b)     blocks until batch b sits in its slot           (returns slot, -1 if stopped)
//   release(b)  the H2D copy of b has completed; slot may be refilled (in-order)
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace {

struct Prefetcher {
  int ntensors = 0, B = 0, R = 0, nthreads = 1;
  std::vector<const char*> host;      // dataset base pointers (row-major, row_bytes[t] per row)
  std::vector<long> row_bytes;
  std::vector<char*> staging;         // staging[t] = R slots of B rows
  std::vector<long> idx;              // epoch's row indices, n_batches * B
  long n_batches = 0;
  long released = 0;                  // batches < released have been consumed
  std::vector<long> slot_batch;       // batch currently valid in each slot (-1 none)
  bool stop = false;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> workers;

  void fill(long b) {
    const int slot = static_cast<int>(b % R);
    for (int t = 0; t < ntensors; ++t) {
      const long rb = row_bytes[t];
      char* dst = staging[t] + static_cast<long>(slot) * B * rb;
      const long* rows = idx.data() + b * B;
      for (int i = 0; i < B; ++i) std::memcpy(dst + i * rb, host[t] + rows[i] * rb, rb);
    }
  }

  void run(int w) {
    for (long b = w; ; b += nthreads) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || b >= n_batches || b < released + R; });
        if (stop || b >= n_batches) return;
      }
      fill(b);
      {
        std::lock_guard<std::mutex> lk(mu);
        slot_batch[b % R] = b;
      }
      cv.notify_all();
    }
  }

  void start(const long* ids, long n_ids, long nb) {
    halt();
    idx.assign(ids, ids + n_ids);
    n_batches = std::min(nb, n_ids / std::max(B, 1));
    released = 0;
    std::fill(slot_batch.begin(), slot_batch.end(), -1L);
    stop = false;
    for (int w = 0; w < nthreads; ++w) workers.emplace_back(&Prefetcher::run, this, w);
  }

  void halt() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& th : workers) th.join();
    workers.clear();
  }

  int wait(long b, long timeout_ms) {
    std::unique_lock<std::mutex> lk(mu);
    auto ok = [&] { return stop || slot_batch[b % R] == b; };
    if (timeout_ms < 0) {
      cv.wait(lk, ok);
    } else if (!cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), ok)) {
      return -2;
    }
    return slot_batch[b % R] == b ? static_cast<int>(b % R) : -1;
  }

  bool ready(long b) {
    std::lock_guard<std::mutex> lk(mu);
    return slot_batch[b % R] == b;
  }

  void release(long b) {
    {
      std::lock_guard<std::mutex> lk(mu);
      released = std::max(released, b + 1);
    }
    cv.notify_all();
  }
};

}  // namespace

extern "C" {

void* mta_prefetch_create(int ntensors, const void* const* host, const long* row_bytes, void* const* staging, int B,
                          int R, int nthreads) {
  auto* p = new Prefetcher();
  p->ntensors = ntensors;
  p->B = B;
  p->R = R;
  p->nthreads = std::max(1, nthreads);
  for (int t = 0; t < ntensors; ++t) {
    p->host.push_back(static_cast<const char*>(host[t]));
    p->row_bytes.push_back(row_bytes[t]);
    p->staging.push_back(static_cast<char*>(staging[t]));
  }
  p->slot_batch.assign(R, -1L);
  return p;
}

void mta_prefetch_start(void* h, const long* idx, long n_idx, long n_batches) {
  static_cast<Prefetcher*>(h)->start(idx, n_idx, n_batches);
}

int mta_prefetch_wait(void* h, long batch, long timeout_ms) { return static_cast<Prefetcher*>(h)->wait(batch, timeout_ms); }

int mta_prefetch_ready(void* h, long batch) { return static_cast<Prefetcher*>(h)->ready(batch) ? 1 : 0; }

void mta_prefetch_release(void* h, long batch) { static_cast<Prefetcher*>(h)->release(batch); }

void mta_prefetch_stop(void* h) { static_cast<Prefetcher*>(h)->halt(); }

void mta_prefetch_destroy(void* h) {
  auto* p = static_cast<Prefetcher*>(h);
  p->halt();
  delete p;
}

}  // extern "C"
