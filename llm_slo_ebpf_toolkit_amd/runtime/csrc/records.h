// Host-side record layouts shared by the native runtime (collector/records.py is the numpy
// mirror; probes/ebpf/mislo_record.h the BPF one; ops/csrc/mislo_common.h the GPU one).
#pragma once

#include <cstdint>

namespace mislo {

struct EventRec {  // records.py EVENT (64 B): the probes' working record, user-space producers' ring record
  int64_t ts_ns;
  uint64_t value;
  uint64_t trace_h;
  uint32_t pid, tid, pod_id, dst_ip;
  uint16_t signal_type, node_id, svc_id, flags, src_port, dst_port;
  int32_t err;
  uint64_t conn_h;
};
static_assert(sizeof(EventRec) == 64, "EVENT is 64 bytes");

struct SpanRec64 {  // records.py SPAN (64 B)
  int64_t ts_ns;
  uint64_t trace_h;
  uint64_t conn_h;
  uint32_t pid, pod_id;
  uint16_t node_id, svc_id;
  uint32_t group_id;
  float ttft_ms, latency_ms;
  uint64_t span_h;
  float retr_ms;  // application-reported retrieval ms (0 = none)
  uint32_t flags;  // bit 0: TTFT-SLO deadline before the agent's last window cut; bit 1: SLI counted
                   // already (first-token record); bit 2: first-token record (SLI only)
};
static_assert(sizeof(SpanRec64) == 64, "SPAN is 64 bytes");

#pragma pack(push, 4)
// records.py SPAN20: what the GPU join reads of a span: absolute timestamp, trace id (same id
// space as the events' trace ids), context id into the device context table, incident group
struct Span20 {
  int64_t ts_ns;
  uint32_t trace_id, ctx_id, group_id;
};
#pragma pack(pop)
static_assert(sizeof(Span20) == 20, "SPAN20 is 20 bytes");

constexpr uint32_t kTsZero = 0xFFFFFFFFu;  // EVENT16 ts_off of a zero timestamp
constexpr int kEpochTagShift = 30;
constexpr uint32_t kTraceIdMask = (1u << kEpochTagShift) - 1u;
// id spaces: the kernel assigns the low half, the agent's host encoder the high half, so
// records from both kinds of producer share one device context table and one trace-id space
constexpr uint32_t kCtxIds = 1u << 24;
constexpr uint32_t kKernelCtxLimit = 1u << 23;   // kernel context ids 1 .. 2^23 - 1
// kernel trace ids 1 .. 2^24 - 1: the probes' LRU trace map (2^20 entries) evicts an idle hash long
// before its id comes round again, and the GPU's id -> hash table stays 128 MiB
constexpr uint32_t kKernelTraceLimit = 1u << 24;

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

// records.py conn32: the 32-bit connection identity carried in context rows (the kernel folds
// the same key in mislo_probe.h mislo_conn32), 0 = no connection
inline uint32_t conn32(uint64_t key) { return key ? ((uint32_t)(key ^ (key >> 32)) | 1u) : 0u; }

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

// records.py milli_shift_table / mislo_record.h mislo_milli_shift: value_milli = raw * 10^d
inline int milli_shift(uint16_t type) {
  switch (type) {
    case 1: case 3: case 4: case 5: case 7: case 8: case 9: case 12: case 13: case 16:
      return -3;  // ns -> ms
    case 6: case 14: case 15:
      return 0;   // milli-percent -> percent, ns -> us
    default:
      return 3;   // counts
  }
}

struct User32Rec {  // records.py USER32
  int64_t ts_ns;
  uint64_t trace_h;
  uint32_t value_milli, pod_id, pid;
  uint8_t signal_type, flags;
  uint16_t node_id;
};
static_assert(sizeof(User32Rec) == 32, "USER32 is 32 bytes");

constexpr uint32_t kUser16TraceBit = 1u << 31;   // records.py USER16_HAS_TRACE
constexpr uint32_t kUser16ContWord = 0xFFFFFFFFu;  // records.py USER16_CONT

struct User24Rec {  // records.py USER24
  uint64_t trace_h;
  uint32_t value_milli, ts_lo;
  uint32_t pid_sig;  // pid | signal_type << 22 | ts_zero << 29 | has_gpu << 30
  uint32_t pod_ts;   // pod_id | (ts bits 32..43) << 20
};
static_assert(sizeof(User24Rec) == 24, "USER24 is 24 bytes");

// records.py to_user: an EVENT as a user-space producer writes it into a `rec`-byte ring (64, 32,
// 24 or 16 bytes at `out`). Returns the slots written: 1, or 2 for a traced USER16 record (its
// continuation slot; `out` must hold two), 0 when the record does not fit USER24 / USER16 (pid >=
// 2^22, pod >= 2^20, signal type >= 128, or 127 in USER16).
inline int pack_user(const EventRec& e, uint32_t rec, void* out) {
  const uint32_t vm = milli_int(e.value, milli_shift(e.signal_type));
  const uint32_t gpu = (e.flags >> 8) & 1u;
  if (rec == 64) {
    *static_cast<EventRec*>(out) = e;
    return 1;
  }
  if (rec == 32) {
    User32Rec u{};
    u.ts_ns = e.ts_ns;
    u.trace_h = e.trace_h;
    u.value_milli = vm;
    u.pod_id = e.pod_id;
    u.pid = e.pid;
    u.signal_type = (uint8_t)e.signal_type;
    u.flags = (uint8_t)gpu;
    u.node_id = e.node_id;
    *static_cast<User32Rec*>(out) = u;
    return 1;
  }
  if ((rec != 24 && rec != 16) || e.pid >= (1u << 22) || e.pod_id >= (1u << 20) || e.signal_type >= 128) return 0;
  if (rec == 16 && e.signal_type >= 127) return 0;
  const uint64_t t = (uint64_t)e.ts_ns;
  User24Rec u{};
  u.trace_h = e.trace_h;
  u.value_milli = vm;
  u.ts_lo = (uint32_t)t;
  u.pid_sig = e.pid | ((uint32_t)e.signal_type << 22) | (e.ts_ns == 0 ? 1u << 29 : 0u) | (gpu << 30);
  u.pod_ts = e.pod_id | (uint32_t)(((t >> 32) & 0xFFFull) << 20);
  if (rec == 24) {
    *static_cast<User24Rec*>(out) = u;
    return 1;
  }
  // USER16: {ts_lo, value, pid_sig | has_trace, pod_ts} [+ {trace lo, trace hi, marker, 0}]
  uint32_t* w = static_cast<uint32_t*>(out);
  w[0] = u.ts_lo;
  w[1] = u.value_milli;
  w[2] = u.pid_sig | (e.trace_h ? kUser16TraceBit : 0u);
  w[3] = u.pod_ts;
  if (!e.trace_h) return 1;
  w[4] = (uint32_t)e.trace_h;
  w[5] = (uint32_t)(e.trace_h >> 32);
  w[6] = kUser16ContWord;
  w[7] = 0u;
  return 2;
}

// EpochClock.stamp (records.py) / mislo_submit: offset of ts from the epoch base
inline uint32_t epoch_offset(int64_t ts, uint64_t base) {
  if (ts == 0) return kTsZero;
  if ((uint64_t)ts < base) return 0;
  const uint64_t d = (uint64_t)ts - base;
  return d >= kTsZero ? kTsZero - 1 : (uint32_t)d;
}

}  // namespace mislo
