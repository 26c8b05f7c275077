#pragma once

#include <atomic>
#include <cstdint>
#include <thread>
#include <vector>

#include "ring.h"

namespace mislo {

class Replayer {
 public:
  Replayer(Ring* ring, const uint8_t* trace, uint64_t n_records, uint32_t rec_size, int64_t lap_ns);
  ~Replayer();
  // rate_eps <= 0: as fast as possible; max_records == 0: until stop()
  void start(int threads, double rate_eps, uint64_t batch, uint64_t max_records);
  void stop();
  void wait();
  bool running() const;
  uint64_t pushed() const { return pushed_.load(); }
  uint64_t dropped() const { return dropped_.load(); }

 private:
  void run(int tid, int nthreads, double rate, uint64_t batch, uint64_t quota);
  Ring* ring_;
  std::vector<uint8_t> trace_;
  uint64_t n_;
  uint32_t rs_;
  int64_t lap_ns_;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> pushed_{0}, dropped_{0};
  std::vector<std::thread> workers_;
};

}  // namespace mislo
