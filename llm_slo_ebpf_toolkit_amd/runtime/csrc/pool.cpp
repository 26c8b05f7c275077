#include "pool.h"

#include <algorithm>
#include <cstring>

namespace mislo {

WorkerPool::WorkerPool(int threads) {
  for (int i = 1; i < std::max(1, threads); ++i) workers_.emplace_back([this] { loop(); });
}

WorkerPool::~WorkerPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void WorkerPool::drain_tasks() {
  for (;;) {
    const int i = next_.fetch_add(1, std::memory_order_relaxed);
    if (i >= ntasks_) return;
    (*fn_)(i);
    std::lock_guard<std::mutex> g(mu_);
    if (--pending_ == 0) done_cv_.notify_all();
  }
}

void WorkerPool::loop() {
  uint64_t seen = 0;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || epoch_ != seen; });
      if (stop_) return;
      seen = epoch_;
    }
    drain_tasks();
  }
}

void WorkerPool::run(int ntasks, const std::function<void(int)>& fn) {
  if (ntasks <= 0) return;
  if (workers_.empty() || ntasks == 1) {
    for (int i = 0; i < ntasks; ++i) fn(i);
    return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    fn_ = &fn;
    ntasks_ = ntasks;
    pending_ = ntasks;
    next_.store(0, std::memory_order_relaxed);
    ++epoch_;
  }
  cv_.notify_all();
  drain_tasks();
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return pending_ == 0; });
  // a worker woken late finds next_ >= ntasks_ and goes back to sleep; fn_ stays valid
  // until the next run() replaces it under the lock
}

void parallel_memcpy(void* dst, const void* src, size_t n, int threads) {
  constexpr size_t kMin = 2u << 20;
  int t = (int)std::min<size_t>((size_t)std::max(1, threads), n / kMin);
  if (t <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> ts;
  const size_t chunk = (n / t + 63) & ~size_t(63);
  for (int i = 1; i < t; ++i) {
    const size_t lo = i * chunk;
    if (lo >= n) break;
    const size_t len = std::min(chunk, n - lo);
    ts.emplace_back([=] { std::memcpy(static_cast<char*>(dst) + lo, static_cast<const char*>(src) + lo, len); });
  }
  std::memcpy(dst, src, std::min(chunk, n));
  for (auto& th : ts) th.join();
}

}  // namespace mislo
