// Host-only building blocks of the native runtime, kept free of HIP / Python so that they
// can be compiled and exercised under the CPU sanitizers (tools/host_selftest.cpp,
// scripts/host_sanitize.sh: AddressSanitizer + UndefinedBehaviorSanitizer and
// ThreadSanitizer builds) -- the GPU sanitizers are not available on this pool.
//
// * OrderedWorker<Job>: one background thread executing submitted jobs strictly in
//   submission order; submit() returns the job's sequence number, wait_issued(seq) blocks
//   until that job (and every earlier one) has run, a job's exception is re-thrown to the
//   waiters.  PinnedPrefetcher (runtime.cpp) runs its slot-reuse wait + pinned memcpy + H2D
//   enqueue on it -- the reference's pin-memory thread (resnet50_test.py:41-43).
// * plan_buckets: DDP gradient bucket assignment (parallel/ddp.py).
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace fdt {

template <class Job>
class OrderedWorker {
 public:
  explicit OrderedWorker(std::function<void(Job&)> fn) : fn_(std::move(fn)) {}
  OrderedWorker(const OrderedWorker&) = delete;
  OrderedWorker& operator=(const OrderedWorker&) = delete;
  ~OrderedWorker() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (thread_.joinable()) thread_.join();  // drains the queue first
  }

  // Queue a job; the worker thread starts on the first submission.
  uint64_t submit(Job j) {
    uint64_t seq;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stop_) throw std::runtime_error("OrderedWorker: submit after shutdown");
      if (!thread_.joinable()) thread_ = std::thread([this] { run(); });
      seq = ++submitted_;
      jobs_.emplace_back(seq, std::move(j));
    }
    cv_.notify_all();
    return seq;
  }

  // Block until job `seq` has run (0: returns at once).  Re-throws the first job error.
  void wait_issued(uint64_t seq) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return done_ >= seq || !error_.empty(); });
    if (!error_.empty()) throw std::runtime_error("background worker: " + error_);
  }
  void drain() {
    uint64_t s;
    {
      std::lock_guard<std::mutex> lk(mu_);
      s = submitted_;
    }
    wait_issued(s);
  }
  uint64_t submitted() const {
    std::lock_guard<std::mutex> lk(mu_);
    return submitted_;
  }
  uint64_t done() const {
    std::lock_guard<std::mutex> lk(mu_);
    return done_;
  }

 private:
  void run() {
    for (;;) {
      std::pair<uint64_t, Job> item;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
        if (jobs_.empty()) return;  // stop requested, queue drained
        item = std::move(jobs_.front());
        jobs_.pop_front();
      }
      std::string err;
      try {
        fn_(item.second);
      } catch (const std::exception& e) {
        err = e.what();
        if (err.empty()) err = "unknown error";
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!err.empty() && error_.empty()) error_ = err;
        done_ = item.first;
      }
      cv_.notify_all();
    }
  }

  std::function<void(Job&)> fn_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<uint64_t, Job>> jobs_;
  uint64_t submitted_ = 0, done_ = 0;
  std::string error_;
  bool stop_ = false;
  std::thread thread_;
};

// sizes: bytes per parameter in REGISTRATION order.  Returns buckets as lists of parameter
// indices, in the order they become ready in backward (reverse registration order): a small
// first bucket (first_cap bytes) so communication starts early in backward, then `cap`.
inline std::vector<std::vector<int>> plan_buckets(const std::vector<size_t>& sizes, size_t first_cap, size_t cap) {
  std::vector<std::vector<int>> buckets;
  std::vector<int> cur;
  size_t acc = 0;
  size_t limit = first_cap;
  for (int i = (int)sizes.size() - 1; i >= 0; --i) {
    cur.push_back(i);
    acc += sizes[(size_t)i];
    if (acc >= limit) {
      buckets.push_back(cur);
      cur.clear();
      acc = 0;
      limit = cap;
    }
  }
  if (!cur.empty()) buckets.push_back(cur);
  return buckets;
}

}  // namespace fdt
