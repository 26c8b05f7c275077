// Native wire encoder: 64-byte EVENT records -> 20-byte EVENT20 / 16-byte EVENT16 wire
// records, written straight into the pinned staging buffer the window is DMA'd from.
//
// The agent-side half of the compact formats (collector/records.py keeps the numpy
// reference implementation the tests compare against):
//   * connection key (conn hash, or the hash of src/dst port + dst ip) -> 24-bit id;
//   * (pod, pid, conn id, svc<<16|node) context -> 24-bit id (append-only table rows that
//     the GPU pipeline uploads once);
//   * EVENT16 only: 64-bit trace hash -> 32-bit id, shared with the spans of the same
//     window so trace equality is exact; ids of traces unseen for two windows are dropped.
// Hash maps are flat open-addressing tables (power-of-two, linear probing, load <= 1/2).
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace mislo {

struct EventRec {  // collector/records.py EVENT (64 B)
  int64_t ts_ns;
  uint64_t value;
  uint64_t trace_h;
  uint32_t pid, tid, pod_id, dst_ip;
  uint16_t signal_type, node_id, svc_id, flags, src_port, dst_port;
  int32_t err;
  uint64_t conn_h;
};
static_assert(sizeof(EventRec) == 64, "EVENT is 64 bytes");

struct SpanRec64 {  // collector/records.py SPAN (64 B)
  int64_t ts_ns;
  uint64_t trace_h;
  uint64_t conn_h;
  uint32_t pid, pod_id;
  uint16_t node_id, svc_id;
  uint32_t group_id;
  float ttft_ms, latency_ms;
  uint64_t span_h, reserved;
};
static_assert(sizeof(SpanRec64) == 64, "SPAN is 64 bytes");

struct Wire20 {
  uint32_t ts_off, ctx_type, value_milli, tr_lo, tr_hi;
};
struct Wire16 {
  uint32_t ts_off, ctx_type, value_milli, trace_id;
};
static_assert(sizeof(Wire20) == 20 && sizeof(Wire16) == 16, "wire record sizes");

constexpr uint32_t kWireTsZero = 0xFFFFFFFFu;

inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// records.py conn_hash_np: 0 when both ports are 0, never 0 otherwise
inline uint64_t conn_key(const EventRec& e) {
  if (e.conn_h) return e.conn_h;
  if (e.src_port == 0 && e.dst_port == 0) return 0;
  const uint64_t packed = ((uint64_t)e.src_port << 48) | ((uint64_t)e.dst_port << 32) | (uint64_t)e.dst_ip;
  const uint64_t h = splitmix64(packed);
  return h ? h : 1;
}

// u64 key (hash) -> u32 value; `eq(value)` resolves hash collisions for composite keys.
class FlatMap {
 public:
  explicit FlatMap(size_t cap = 1024);
  template <class Eq>
  uint32_t* find(uint64_t h, Eq eq);
  void insert(uint64_t h, uint32_t v);
  size_t size() const { return size_; }
  void clear();

 private:
  void grow();
  std::vector<uint64_t> keys_;  // 0 = empty slot (stored hashes are forced non-zero)
  std::vector<uint32_t> vals_;
  size_t mask_ = 0, size_ = 0;
};

// trace hash -> 32-bit id with the generation (window) of last use; entries unused for two
// generations are dropped when the table is rebuilt, so memory stays bounded.
class TraceTable {
 public:
  TraceTable();
  uint32_t id(uint64_t tr, uint32_t gen);
  void expire(uint32_t min_gen);
  size_t size() const { return size_; }

 private:
  void rehash(size_t cap, uint32_t min_gen);
  std::vector<uint64_t> keys_;
  std::vector<uint32_t> ids_, gens_;
  size_t mask_ = 0, size_ = 0;
  uint32_t next_ = 1;
};

class WireEncoder {
 public:
  // scale[t]: raw kernel value -> output unit for signal type t < 256 (catalog.decode_scale)
  explicit WireEncoder(const double* scale256);

  // Encodes n events into `out` (wire 20 or 16). Returns t_base (earliest non-zero ts).
  // Throws std::range_error if the window spans >= 2^32 - 1 ns.
  int64_t encode(const EventRec* ev, size_t n, void* out, int wire);
  // Spans keep the 64-byte layout: conn hash -> conn id; with trace_ids, trace -> id.
  void encode_spans(const SpanRec64* in, size_t n, SpanRec64* out, bool trace_ids);
  // Trace-id generation boundary (call once per window after events and spans).
  void end_window();

  const std::vector<std::array<uint32_t, 4>>& ctx_rows() const { return ctx_rows_; }
  size_t n_conns() const { return n_conns_; }
  size_t n_traces() const { return traces_.size(); }
  uint32_t generation() const { return gen_; }

 private:
  uint32_t conn_id(uint64_t key);
  uint32_t ctx_id(uint32_t pod, uint32_t pid, uint32_t cid, uint32_t sn);

  double scale_[256];
  FlatMap conns_{1 << 12};
  size_t n_conns_ = 0;
  FlatMap ctx_{1 << 12};
  std::vector<std::array<uint32_t, 4>> ctx_rows_;
  TraceTable traces_;
  uint32_t gen_ = 1;
};

}  // namespace mislo
