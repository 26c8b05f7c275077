// User-space model of the probes' in-kernel record path (probes/ebpf/mislo_probe.h
// mislo_submit), for the tests, the CPU-only CI and the benchmark's producer, which cannot
// load BPF (no BPF target in the toolchain, no root on the GPU pool).
//
// Given the 64-byte working record a probe fills (mislo_reserve), it does what the BPF program
// does, in the same order:
//   * fixed-point value (mislo_milli), 32-bit connection identity (mislo_conn32);
//   * context (pod, pid, conn32) -> id from the mislo_ctxs map, a fresh id drawn from counter
//     mislo_cfg[126] on first sight, its definition record (mislo_def16 CTX) committed to the
//     ring BEFORE the id is inserted, so no event can reference an id whose definition is not
//     ahead of it in ring order;
//   * trace hash -> id from the mislo_traces LRU map, same protocol (TRACE definitions);
//   * timestamp as an offset from the epoch the agent published in mislo_cfg[124], tagged;
//   * bpf_ringbuf_output of the 16-byte record.
// Thread-safe (the maps sit behind a mutex; the ring's own lock orders reservations).
#pragma once

#include <cstdint>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "bpfring.h"
#include "records.h"

namespace mislo {

constexpr int kCfgClock = 0, kCfgNode = 1, kCfgEpoch = 124, kCfgTraceNext = 125, kCfgCtxNext = 126;
inline int cfg_floor(int type) { return 2 + type; }

class ProbeSim {
 public:
  // cfg: the emulated mislo_cfg array (kCfgSlots u64, e.g. Ringbuf::cfg()); shift256: records.py
  // milli_shift_table
  ProbeSim(uint64_t* cfg, const int8_t* shift256, size_t trace_lru = 1u << 20);
  // every record through mislo_emit: floors checked, defs + event output into `rb`; returns the
  // number of event records committed (a full ring drops, as bpf_ringbuf_output does)
  uint64_t submit(Ringbuf& rb, const EventRec* ev, size_t n);
  // the same records as ring payloads, appended to `out` (an image for append_framed)
  void encode(const EventRec* ev, size_t n, std::vector<Rec16>& out);
  uint64_t dropped() const { return dropped_; }
  size_t n_ctx() const { return ctx_.size(); }
  size_t n_traces() const { return traces_.size(); }
  // what the agent does when the id space runs low: clear the maps and counters
  void reset_maps();

 private:
  template <class Emit>
  void one(const EventRec& e, Emit&& emit);
  uint64_t* cfg_;
  int8_t shift_[256];
  size_t trace_lru_;
  std::mutex mu_;
  std::unordered_map<uint64_t, uint32_t> traces_;
  struct CtxKey {
    uint32_t pod, pid, c32;
    bool operator==(const CtxKey& o) const { return pod == o.pod && pid == o.pid && c32 == o.c32; }
  };
  struct CtxHash {
    size_t operator()(const CtxKey& k) const { return (size_t)splitmix64(((uint64_t)k.pod << 32 | k.pid) ^ k.c32); }
  };
  std::unordered_map<CtxKey, uint32_t, CtxHash> ctx_;
  uint64_t dropped_ = 0;
};

}  // namespace mislo
