// CPU self-test of the host-only runtime pieces (csrc/runtime/ordered_worker.h), built by
// scripts/host_sanitize.sh under AddressSanitizer + UndefinedBehaviorSanitizer and under
// ThreadSanitizer (SURVEY.md §5 race detection; the GPU sanitizers are not available on this
// pool).  Exit status 0 = every check passed and no sanitizer report.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <vector>

#include "../csrc/runtime/ordered_worker.h"

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                  \
    }                                                                \
  } while (0)

static void test_plan_buckets() {
  using fdt::plan_buckets;
  CHECK(plan_buckets({}, 10, 10).empty());
  auto b = plan_buckets({4, 4, 4, 4, 4}, 4, 8);  // first bucket = last param alone, then 8 B
  CHECK(b.size() == 3 && b[0] == std::vector<int>({4}) && b[1] == std::vector<int>({3, 2}) &&
        b[2] == std::vector<int>({1, 0}));
  // every index exactly once, in reverse registration order
  std::vector<size_t> sizes(1000);
  for (size_t i = 0; i < sizes.size(); ++i) sizes[i] = (i * 7919) % 4096 + 1;
  auto bb = plan_buckets(sizes, 1 << 12, 1 << 16);
  int expect = (int)sizes.size() - 1;
  for (auto& v : bb)
    for (int i : v) CHECK(i == expect--);
  CHECK(expect == -1);
  // zero-size parameters never make a bucket boundary on their own
  auto z = plan_buckets({0, 0, 0}, 1, 1);
  CHECK(z.size() == 1 && z[0].size() == 3);
}

struct CopyJob {
  int slot;
  const std::vector<unsigned char>* src;
};

static void test_worker_ring() {
  // the PinnedPrefetcher pattern: a ring of 3 "pinned" slots filled by the worker, read by
  // the submitting thread after wait_issued (the happens-before the sanitizer checks)
  constexpr int kSlots = 3, kBytes = 1 << 16, kJobs = 200;
  std::vector<std::vector<unsigned char>> ring(kSlots, std::vector<unsigned char>(kBytes));
  std::vector<std::vector<unsigned char>> srcs(kJobs, std::vector<unsigned char>(kBytes));
  for (int k = 0; k < kJobs; ++k) std::memset(srcs[k].data(), k & 0xff, kBytes);
  std::vector<int> order;  // touched by the worker only until drained
  {
    fdt::OrderedWorker<CopyJob> w([&](CopyJob& j) {
      std::memcpy(ring[j.slot].data(), j.src->data(), kBytes);
      order.push_back(j.slot);
    });
    std::vector<uint64_t> seq(kSlots, 0);
    for (int k = 0; k < kJobs; ++k) {
      const int s = k % kSlots;
      if (k >= kSlots) {  // the slot's previous batch is consumed before it is refilled
        w.wait_issued(seq[s]);
        const unsigned char want = (unsigned char)((k - kSlots) & 0xff);
        for (int i = 0; i < kBytes; i += 4093) CHECK(ring[s][i] == want);
      }
      seq[s] = w.submit(CopyJob{s, &srcs[k]});
      CHECK(seq[s] == (uint64_t)k + 1);
    }
    w.drain();
    CHECK(w.done() == (uint64_t)kJobs && w.submitted() == (uint64_t)kJobs);
  }
  CHECK((int)order.size() == kJobs);
  for (int k = 0; k < kJobs; ++k) CHECK(order[k] == k % kSlots);
}

static void test_worker_errors_and_shutdown() {
  std::atomic<int> ran{0};
  {
    fdt::OrderedWorker<int> w([&](int& v) {
      ran++;
      if (v == 5) throw std::runtime_error("job 5 failed");
    });
    for (int i = 0; i < 10; ++i) w.submit(i);
    bool threw = false;
    try {
      w.drain();
    } catch (const std::runtime_error& e) {
      threw = std::strstr(e.what(), "job 5 failed") != nullptr;
    }
    CHECK(threw);
  }  // destructor drains the remaining jobs and joins
  CHECK(ran == 10);
  {
    fdt::OrderedWorker<int> idle([](int&) {});  // never started: destructor must not hang
    idle.wait_issued(0);
  }
  {
    // shutdown with work still queued
    std::atomic<long> sum{0};
    {
      fdt::OrderedWorker<int> w([&](int& v) { sum += v; });
      for (int i = 0; i < 5000; ++i) w.submit(i);
    }
    CHECK(sum == 5000L * 4999 / 2);
  }
}

int main() {
  test_plan_buckets();
  test_worker_ring();
  test_worker_errors_and_shutdown();
  std::printf("host_selftest: ok\n");
  return 0;
}
