// Engine host staging pool (see staging.cpp for the Python binding and the design notes):
// persistent copy threads gather a batch of per-request buffers into one pinned slot.  Header-only
// so the same code is built into the pybind11 module and into tests/native/staging_sanitize.cpp
// (ThreadSanitizer / AddressSanitizer, no Python).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

namespace mls_staging {


constexpr size_t kChunk = 256 * 1024;

struct Job {
  char* dst = nullptr;
  std::vector<const char*> srcs;
  size_t each = 0;        // bytes per request
  size_t chunks_per = 0;  // chunks per request
  size_t total = 0;       // chunks in the job
  std::atomic<size_t> next{0};
  std::atomic<size_t> done{0};
};

class Stager {
 public:
  explicit Stager(int threads) {
    if (threads < 0) throw std::invalid_argument("threads must be >= 0");
    for (int i = 0; i < threads; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~Stager() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

  int threads() const { return static_cast<int>(workers_.size()); }

  // Copy srcs[i] (each `each` bytes) to dst + i * each.  Blocks until every byte is written.
  void gather(uintptr_t dst, const std::vector<uintptr_t>& srcs, size_t each) {
    if (srcs.empty() || each == 0) return;
    std::lock_guard<std::mutex> one(call_mu_);  // one batch at a time per stager
    bool wake = false;
    {
      // the job is rewritten only while no worker is inside work(): a worker that woke late for
      // the previous batch (and found its chunks exhausted) may still be reading the counters
      std::unique_lock<std::mutex> g(mu_);
      idle_cv_.wait(g, [this] { return active_ == 0; });
      job_.dst = reinterpret_cast<char*>(dst);
      job_.srcs.resize(srcs.size());
      for (size_t i = 0; i < srcs.size(); ++i) job_.srcs[i] = reinterpret_cast<const char*>(srcs[i]);
      job_.each = each;
      job_.chunks_per = (each + kChunk - 1) / kChunk;
      job_.total = job_.chunks_per * srcs.size();
      job_.next.store(0, std::memory_order_relaxed);
      job_.done.store(0, std::memory_order_relaxed);
      wake = !workers_.empty() && job_.total > 1;
      if (wake) ++gen_;
    }
    if (wake) cv_.notify_all();
    work();  // the caller copies too
    // every chunk written (release/acquire on `done`); late workers only see an exhausted cursor
    while (job_.done.load(std::memory_order_acquire) < job_.total) std::this_thread::yield();
  }

 private:
  void work() {
    const size_t total = job_.total;  // stable while this thread is counted in active_
    for (;;) {
      size_t c = job_.next.fetch_add(1, std::memory_order_relaxed);
      if (c >= total) return;
      size_t req = c / job_.chunks_per, part = c % job_.chunks_per;
      size_t off = part * kChunk;
      size_t n = job_.each - off < kChunk ? job_.each - off : kChunk;
      std::memcpy(job_.dst + req * job_.each + off, job_.srcs[req] + off, n);
      job_.done.fetch_add(1, std::memory_order_release);
    }
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        ++active_;
      }
      work();
      {
        std::lock_guard<std::mutex> g(mu_);
        --active_;
      }
      idle_cv_.notify_all();
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_, idle_cv_;
  uint64_t gen_ = 0;
  int active_ = 0;
  bool stop_ = false;
  Job job_;
};

}  // namespace mls_staging
