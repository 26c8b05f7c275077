// Paced replay producers: N threads push a pre-generated record trace into a Ring at a
// target aggregate rate (events/s), looping over the trace with timestamps shifted
// forward on every lap so the stream stays monotonic -- the stand-in for kernel probes
// (BPF ring-buffer readers) and the rocprofiler-sdk tool when measuring the agent's
// throughput and CPU overhead on a host without BPF privileges.
#include "replay.h"

#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

namespace mislo {

namespace {
inline void shift_ts(uint8_t* rec, uint32_t rec_size, int64_t delta) {
  if (rec_size == 64) {  // EVENT / SPAN: ts_ns at offset 0
    int64_t ts;
    std::memcpy(&ts, rec, 8);
    ts += delta;
    std::memcpy(rec, &ts, 8);
  } else if (rec_size == 40) {  // REF record: timestamp_ns at offset 8
    uint64_t ts;
    std::memcpy(&ts, rec + 8, 8);
    ts += (uint64_t)delta;
    std::memcpy(rec + 8, &ts, 8);
  }
}
}  // namespace

Replayer::Replayer(Ring* ring, const uint8_t* trace, uint64_t n_records, uint32_t rec_size, int64_t lap_ns)
    : ring_(ring), trace_(trace, trace + n_records * rec_size), n_(n_records), rs_(rec_size), lap_ns_(lap_ns) {}

Replayer::~Replayer() { stop(); }

void Replayer::start(int threads, double rate_eps, uint64_t batch, uint64_t max_records) {
  stop();
  stop_.store(false);
  pushed_.store(0);
  dropped_.store(0);
  if (threads < 1) threads = 1;
  if (batch < 1) batch = 1;
  for (int t = 0; t < threads; ++t) {
    workers_.emplace_back([this, t, threads, rate_eps, batch, max_records] {
      run(t, threads, rate_eps / threads, batch, max_records == 0 ? 0 : (max_records + threads - 1) / threads);
    });
  }
}

void Replayer::run(int tid, int nthreads, double rate, uint64_t batch, uint64_t quota) {
  std::vector<uint8_t> buf(batch * rs_);
  // each thread replays an interleaved stripe of the trace
  uint64_t cursor = (uint64_t)tid * batch, lap = 0, done = 0;
  const auto t0 = std::chrono::steady_clock::now();
  while (!stop_.load(std::memory_order_relaxed)) {
    if (quota && done >= quota) break;
    uint64_t nb = batch;
    if (quota && done + nb > quota) nb = quota - done;
    for (uint64_t i = 0; i < nb; ++i) {
      uint64_t r = cursor + i;
      uint64_t l = lap + r / n_;
      r %= n_;
      std::memcpy(buf.data() + i * rs_, trace_.data() + r * rs_, rs_);
      if (l) shift_ts(buf.data() + i * rs_, rs_, (int64_t)l * lap_ns_);
    }
    cursor += (uint64_t)nthreads * batch;
    if (cursor >= n_) {
      lap += cursor / n_;
      cursor %= n_;
    }
    const uint64_t ok = ring_->push_batch(buf.data(), nb);
    if (ok) pushed_.fetch_add(ok, std::memory_order_relaxed);
    else dropped_.fetch_add(nb, std::memory_order_relaxed);
    done += nb;
    if (rate > 0) {  // pace: sleep until this thread's schedule catches up
      const double due_s = (double)done / rate;
      const auto due = t0 + std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                std::chrono::duration<double>(due_s));
      std::this_thread::sleep_until(due);
    }
  }
}

void Replayer::stop() {
  stop_.store(true);
  for (auto& w : workers_)
    if (w.joinable()) w.join();
  workers_.clear();
}

bool Replayer::running() const {
  for (auto& w : workers_)
    if (w.joinable()) return true;
  return false;
}

void Replayer::wait() {
  for (auto& w : workers_)
    if (w.joinable()) w.join();
  workers_.clear();
}

}  // namespace mislo
