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
//
// encode_window() is the agent's hot path: one window's events and spans in three phases on a
// worker pool, byte-identical to encode() + encode_spans() run sequentially:
//   1. parallel over contiguous chunks: fixed-point values and provisional timestamps; every
//      key is looked up in the (read-only) global tables; keys not there yet go to a chunk-
//      local first-seen list and the record holds the local index, noted in a fix-up list;
//   2. serial: the chunks' new-key lists are merged in chunk order, which is global first-
//      occurrence order, so ids come out exactly as the sequential encoder assigns them;
//   3. parallel: fix-up records get their global ids (and timestamps are rebased in the rare
//      window whose first event is not its earliest).
#pragma once

#include <array>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
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
struct Event24 {  // collector/records.py EVENT24 = probes/ebpf/mislo_record.h mislo_event24
  int64_t ts_ns;
  uint64_t trace_h;
  uint32_t value_milli, ctx_type;
};
static_assert(sizeof(Event24) == 24, "Event24 is 24 bytes");

#pragma pack(push, 4)
// records.py SPAN20: a span as the GPU join needs it (20 B instead of 64): absolute timestamp,
// interned trace id, (pod, pid, conn, svc|node) context id into the device context table,
// incident group
struct Span20 {
  int64_t ts_ns;
  uint32_t trace_id, ctx_id, group_id;
};
struct Event20T {  // collector/records.py EVENT20T = probes/ebpf/mislo_record.h mislo_event20t (wire code 21)
  int64_t ts_ns;
  uint32_t value_milli, ctx_type, trace_id;
};
#pragma pack(pop)
static_assert(sizeof(Event20T) == 20 && sizeof(Span20) == 20, "Event20T / Span20 are 20 bytes");
constexpr int kWire20T = 21;
inline int wire_bytes(int wire) { return wire == kWire20T ? 20 : wire; }

struct Event32 {  // collector/records.py EVENT32 = probes/ebpf/mislo_record.h mislo_event32
  int64_t ts_ns;
  uint64_t trace_h;
  uint32_t value_milli, pid, pod_id, type_conn;
};
static_assert(sizeof(Wire20) == 20 && sizeof(Wire16) == 16 && sizeof(Event32) == 32, "wire record sizes");

// records.py milli_int: v * 10^d rounded half-to-even, saturated to u32 (integer-only, the
// same rule the BPF probes apply in the kernel)
inline uint32_t milli_int(uint64_t v, int d) {
  static constexpr uint64_t kP10[10] = {1ull,      10ull,      100ull,      1000ull,      10000ull,
                                        100000ull, 1000000ull, 10000000ull, 100000000ull, 1000000000ull};
  constexpr uint64_t kLim = 0xFFFFFFFFull;
  if (d >= 0) {
    const uint64_t p = kP10[d];
    if (v > kLim / p) return (uint32_t)kLim;
    return (uint32_t)(v * p);
  }
  uint64_t q, r, p;
  if (d == -3) {  // ns -> ms: the common case, constant divisor
    q = v / 1000, r = v % 1000, p = 1000;
  } else {
    p = kP10[-d], q = v / p, r = v % p;
  }
  q += (2 * r > p) || (2 * r == p && (q & 1));
  return q > kLim ? (uint32_t)kLim : (uint32_t)q;
}

constexpr uint32_t kWireTsZero = 0xFFFFFFFFu;
// EVENT16 trace_id: bits 0-29 interned trace id, bits 30-31 the epoch tag (which of the
// window's 4 timestamp bases ts_off counts from; the host encoder writes tag 0)
constexpr int kEpochTagShift = 30;
constexpr uint32_t kTraceIdMask = (1u << kEpochTagShift) - 1u;

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
  // read-only lookup for concurrent readers: id or 0 if absent; marks the entry used in `gen`
  // (a relaxed store, only when it changes)
  uint32_t find_touch(uint64_t tr, uint32_t gen);
  void expire(uint32_t min_gen);
  size_t size() const { return size_; }

 private:
  void rehash(size_t cap, uint32_t min_gen);
  struct Slot {  // one cache access per probe
    uint64_t key;
    uint32_t id, gen;
  };
  std::vector<Slot> slots_;
  size_t mask_ = 0, size_ = 0;
  uint32_t next_ = 1;
};

// (pod<<32|pid, conn key, svc<<16|node) -> id with the key stored in the slot (one cache
// access per probe; no side table to compare against). id kEmpty marks a free slot.
class CtxMap {
 public:
  static constexpr uint32_t kEmpty = 0xFFFFFFFFu;
  explicit CtxMap(size_t cap = 64);
  uint32_t find(uint64_t h, uint64_t ppid, uint64_t ck, uint32_t sn) const;  // kEmpty if absent
  void insert(uint64_t h, uint64_t ppid, uint64_t ck, uint32_t sn, uint32_t id);
  size_t size() const { return size_; }
  void clear();

 private:
  struct Slot {
    uint64_t ppid, ck, h;
    uint32_t sn, id;
  };
  std::vector<Slot> slots_;
  size_t mask_ = 0, size_ = 0;
};

// Fixed pool of worker threads; run(n, fn) executes fn(0..n-1) on the workers and the calling
// thread and returns when all are done. Idle workers block on a condition variable (no
// spinning: the agent's CPU budget is measured).
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

// Per-chunk scratch of encode_window (reused across windows).
struct ChunkScratch {
  int64_t tmin, tmax;
  FlatMap conn_map{64}, trace_map{256};
  CtxMap ctx_map{64};
  std::vector<uint64_t> new_conns, new_traces;
  std::vector<std::array<uint64_t, 3>> new_ctx;  // pod<<32|pid, conn key, svc<<16|node
  std::vector<uint64_t> fix;                     // record index << 2 | (1: ctx / conn, 2: trace)
  std::vector<uint32_t> conn_remap, ctx_remap, trace_remap;
  void reset();
};

class WireEncoder {
 public:
  // shift[t]: value_milli = raw * 10^shift[t] for signal type t < 256 (records.py
  // milli_shift_table; types >= 256 use 3)
  explicit WireEncoder(const int8_t* shift256);

  // Encodes n events into `out` (wire 20 or 16). Returns t_base (earliest non-zero ts).
  // Throws std::range_error if the window spans >= 2^32 - 1 ns. wire 32 / 24 / 21 write Event32 /
  // Event24 / Event20T (the records the probes emit: absolute ts; interned connection / context
  // ids; Event20T also interned trace ids, shared with encode_spans(trace_ids = true)) and
  // return 0.
  int64_t encode(const EventRec* ev, size_t n, void* out, int wire);
  // Spans keep the 64-byte layout: conn hash -> conn id; with trace_ids, trace -> id.
  void encode_spans(const SpanRec64* in, size_t n, SpanRec64* out, bool trace_ids);
  // Spans -> Span20 (trace ids and contexts on the same tables as the events; new contexts
  // append ctx rows like events do)
  void encode_spans20(const SpanRec64* in, size_t n, Span20* out);
  // Trace-id generation boundary (call once per window after events and spans).
  void end_window();
  // events -> ev_out (wire 20/16) and spans -> sp_out in one pass on `threads` threads; the
  // same bytes and ids as encode() then encode_spans(ev_out, trace_ids = wire == 16). Does not
  // call end_window(). Throws std::range_error (tables untouched) like encode().
  int64_t encode_window(const EventRec* ev, size_t n, void* ev_out, int wire, const SpanRec64* sp, size_t n_sp,
                        SpanRec64* sp_out, int threads, size_t min_chunk = 16384);

  const std::vector<std::array<uint32_t, 4>>& ctx_rows() const { return ctx_rows_; }
  size_t n_conns() const { return n_conns_; }
  size_t n_traces() const { return traces_.size(); }
  uint32_t generation() const { return gen_; }

 private:
  uint32_t conn_id(uint64_t key);
  uint32_t conn_find(uint64_t key);  // read-only: 0 if absent (key != 0)
  // contexts are keyed by the connection KEY (a bijection with its id), so chunks can test a
  // context for novelty before new connections have ids
  uint32_t ctx_id(uint32_t pod, uint32_t pid, uint64_t ckey, uint32_t sn);
  uint32_t ctx_find(uint32_t pod, uint32_t pid, uint64_t ckey, uint32_t sn);  // read-only: kAbsent
  static constexpr uint32_t kAbsent = CtxMap::kEmpty;
  void encode_chunk(const EventRec* ev, size_t lo, size_t hi, int64_t base, void* out, int wire, ChunkScratch& cs);
  void spans_chunk(const SpanRec64* sp, size_t lo, size_t hi, SpanRec64* out, bool trace_ids, ChunkScratch& cs);

  int8_t shift_[256];
  FlatMap conns_{1 << 12};
  size_t n_conns_ = 0;
  CtxMap ctx_{1 << 12};
  std::vector<std::array<uint32_t, 4>> ctx_rows_;
  std::unique_ptr<WorkerPool> pool_;
  std::vector<ChunkScratch> chunks_;
  TraceTable traces_;
  uint32_t gen_ = 1;
};

}  // namespace mislo
