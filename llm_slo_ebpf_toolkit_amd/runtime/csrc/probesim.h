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
//   * the 16-byte slot into the CPU's staging batch (mislo_stage_put): a batch goes on the ring
//     as one 136-byte record when its 8 slots are full, when a definition joins it (a definition
//     is on the ring before its id is in the map), before a slot of a newer epoch joins it, and
//     at the agent's window cut (flush(): every CPU's batch, CPU 0 first; unused slots are pads).
// A task's CPU is modelled as tid % cpus. Thread-safe (maps and batches behind a mutex; the
// ring's own lock orders reservations).
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
  ProbeSim(uint64_t* cfg, const int8_t* shift256, size_t trace_lru = 1u << 20, uint32_t cpus = 16);
  // every record through mislo_emit: floors checked, defs + event slots staged, full batches
  // output into `rb`, and with `flush` the partial batches too (the agent's cut); returns the
  // number of events committed to the ring by this call (a full ring drops a whole batch, as
  // bpf_ringbuf_output does)
  uint64_t submit(Ringbuf& rb, const EventRec* ev, size_t n, bool flush = true);
  uint64_t flush(Ringbuf& rb);
  // the same records as ring payloads (whole batches of 8 slots), appended to `out` (an image for
  // append_framed); encode_flush appends the partial batches
  void encode(const EventRec* ev, size_t n, std::vector<Rec16>& out, bool flush = true);
  void encode_flush(std::vector<Rec16>& out);
  uint64_t dropped() const { return dropped_; }  // events lost to a full ring
  uint64_t batches() const { return batches_; }  // batches output (ring records)
  size_t n_ctx() const { return ctx_.size(); }
  size_t n_traces() const { return traces_.size(); }
  // what the agent does when the id space runs low: clear the maps and counters
  void reset_maps();

 private:
  struct Stage {
    uint32_t n = 0;
    uint64_t epoch = 0;
    Rec16 slot[kBatchSlots];
  };
  // mislo_stage_put: returns false when the batch carrying `r` could not go on the ring (only
  // meaningful for definitions, which flush at once)
  template <class Out>
  bool put(uint32_t cpu, const Rec16& r, bool def, Out&& out);
  template <class Out>
  bool flush_stage(Stage& st, Out&& out);
  template <class Out>
  void one(const EventRec& e, Out&& out);
  uint64_t* cfg_;
  int8_t shift_[256];
  size_t trace_lru_;
  std::vector<Stage> stages_;
  uint64_t batches_ = 0;
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
