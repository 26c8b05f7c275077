// Fixed pool of worker threads for the agent's per-window host work (ring compaction, host
// record encoding). run(n, fn) executes fn(0..n-1) on the workers and the calling thread and
// returns when all are done. Idle workers block on a condition variable (no spinning: the
// agent's CPU budget is measured, REF pkg/safety/overhead_guard.go:77-107).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace mislo {

class WorkerPool {
 public:
  explicit WorkerPool(int threads);
  ~WorkerPool();
  void run(int ntasks, const std::function<void(int)>& fn);
  int threads() const { return (int)workers_.size() + 1; }

 private:
  void loop();
  void drain_tasks();
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int ntasks_ = 0;
  std::atomic<int> next_{0};
  int pending_ = 0;  // tasks not finished (guarded by mu_)
  uint64_t epoch_ = 0;
  bool stop_ = false;
};

// memcpy of a large block split over `threads` short-lived threads (>= 2 MiB per thread);
// producers use it for bulk appends, which a single core's memcpy bandwidth would bound
void parallel_memcpy(void* dst, const void* src, size_t n, int threads);

}  // namespace mislo
