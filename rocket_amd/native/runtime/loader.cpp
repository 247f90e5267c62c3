// Native host batch assembler (DataLoader + blocking H2D copy).
//
// For datasets held in host memory as aligned row-major arrays (images, labels, ...), a batch is
// a row gather.  Python worker processes and per-sample collate are replaced by a pool of C++
// threads that copy the selected rows of every tensor straight into a PINNED staging buffer;
// the Python side then issues one non_blocking H2D copy per tensor on a copy stream.  Jobs are
// asynchronous: submit(slot) returns immediately, wait(slot) blocks until that slot's rows are
// in place, so batch k+1 is assembled while batch k is copied and batch k-1 computes.
//
// Work split: a job of n rows is cut into chunks of >= 64 rows (or ~n/threads) that the pool
// threads pull from a shared counter; each chunk copies its rows for all tensors (memcpy per
// row: rows are hundreds of bytes to a few KB, well above memcpy's small-size overhead).
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#define RKL_API extern "C" __attribute__((visibility("default")))

namespace {

struct Job {
  std::vector<int64_t> idx;
  std::vector<char*> dst;
  std::atomic<int64_t> next{0};
  std::atomic<int64_t> done{0};
  int64_t chunk = 64;
};

struct Slot {
  std::shared_ptr<Job> job;
  std::mutex m;
  std::condition_variable cv;
  bool busy = false;
};

struct Loader {
  std::vector<const char*> base;
  std::vector<int64_t> row_bytes;
  int64_t nrows = 0;
  std::vector<std::thread> threads;
  std::deque<std::pair<std::shared_ptr<Job>, Slot*>> queue;
  std::mutex qm;
  std::condition_variable qcv;
  bool stop = false;
  std::vector<Slot> slots;

  void run_chunks(const std::shared_ptr<Job>& j, Slot* s) {
    const int64_t n = (int64_t)j->idx.size();
    for (;;) {
      const int64_t c0 = j->next.fetch_add(j->chunk);
      if (c0 >= n) break;
      const int64_t c1 = c0 + j->chunk < n ? c0 + j->chunk : n;
      for (size_t t = 0; t < base.size(); ++t) {
        const int64_t rb = row_bytes[t];
        char* d = j->dst[t];
        const char* b = base[t];
        for (int64_t r = c0; r < c1; ++r) {
          int64_t src = j->idx[r];
          if (src < 0) src += nrows;
          std::memcpy(d + r * rb, b + src * rb, (size_t)rb);
        }
      }
      if (j->done.fetch_add(c1 - c0) + (c1 - c0) == n) {
        std::lock_guard<std::mutex> g(s->m);
        s->busy = false;
        s->cv.notify_all();
      }
    }
  }

  void worker() {
    for (;;) {
      std::pair<std::shared_ptr<Job>, Slot*> item;
      {
        std::unique_lock<std::mutex> g(qm);
        qcv.wait(g, [&] { return stop || !queue.empty(); });
        if (stop && queue.empty()) return;
        item = queue.front();
        // leave the job queued while chunks remain so every idle thread can help
        if (item.first->next.load() >= (int64_t)item.first->idx.size()) {
          queue.pop_front();
          continue;
        }
      }
      run_chunks(item.first, item.second);
      std::lock_guard<std::mutex> g(qm);
      if (!queue.empty() && queue.front().first == item.first) queue.pop_front();
    }
  }
};

}  // namespace

RKL_API int rkl_create(void** out, int ntensors, const void* const* bases, const int64_t* row_bytes, int64_t nrows,
                       int nthreads, int nslots) {
  Loader* L = new Loader();
  for (int i = 0; i < ntensors; ++i) {
    L->base.push_back((const char*)bases[i]);
    L->row_bytes.push_back(row_bytes[i]);
  }
  L->nrows = nrows;
  L->slots = std::vector<Slot>(nslots > 0 ? nslots : 1);
  if (nthreads < 1) nthreads = 1;
  for (int t = 0; t < nthreads; ++t) L->threads.emplace_back([L] { L->worker(); });
  *out = L;
  return 0;
}

// queue the gather of rows idx[0..n) into dsts[t] (each >= n * row_bytes[t] bytes) on `slot`
RKL_API int rkl_submit(void* loader, int slot, const int64_t* idx, int64_t n, void* const* dsts) {
  Loader* L = (Loader*)loader;
  if (slot < 0 || slot >= (int)L->slots.size()) return 1;
  Slot& s = L->slots[slot];
  {
    std::unique_lock<std::mutex> g(s.m);
    s.cv.wait(g, [&] { return !s.busy; });  // a slot's previous job must be finished
    s.busy = n > 0;
  }
  if (n <= 0) return 0;
  auto j = std::make_shared<Job>();
  j->idx.assign(idx, idx + n);
  for (size_t t = 0; t < L->base.size(); ++t) j->dst.push_back((char*)dsts[t]);
  const int64_t per = (n + (int64_t)L->threads.size() - 1) / (int64_t)L->threads.size();
  j->chunk = per < 64 ? 64 : per;
  s.job = j;
  {
    std::lock_guard<std::mutex> g(L->qm);
    L->queue.emplace_back(j, &s);
  }
  L->qcv.notify_all();
  return 0;
}

RKL_API int rkl_wait(void* loader, int slot) {
  Loader* L = (Loader*)loader;
  if (slot < 0 || slot >= (int)L->slots.size()) return 1;
  Slot& s = L->slots[slot];
  std::unique_lock<std::mutex> g(s.m);
  s.cv.wait(g, [&] { return !s.busy; });
  return 0;
}

RKL_API int rkl_destroy(void* loader) {
  Loader* L = (Loader*)loader;
  if (!L) return 0;
  for (size_t i = 0; i < L->slots.size(); ++i) rkl_wait(L, (int)i);
  {
    std::lock_guard<std::mutex> g(L->qm);
    L->stop = true;
  }
  L->qcv.notify_all();
  for (auto& t : L->threads) t.join();
  delete L;
  return 0;
}
