// Shared device/host definitions for the MI355X (gfx950) LLM-SLO engine kernels.
//
// Record layouts mirror llm_slo_ebpf_toolkit_amd/collector/records.py (EVENT, SPAN,
// REF_EVENT). Signal slots / decode scales / thresholds / histogram edges mirror
// signals/catalog.py and are uploaded once into __constant__ memory (mislo_set_tables).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mislo {

constexpr int kSlots = 16;          // feature slots (12 REF + 4 GPU signals)
constexpr int kBuckets = 16;        // histogram buckets per slot (15 edges + overflow)
constexpr int kKeyTypes = 4;        // trace, pod+pid, pod+conn, svc+node
// Hash partitions per key type. Fewer, larger partitions make the scatter's per-(workgroup,
// partition) runs longer (2^7: scatter 71 -> 41 us per halo-on window) but every probe item
// stages and searches a bigger span chunk (2^7: probe 217 -> 258 us); 2^10 is the better total
// on MI355X (profiles/r3_prof/kernel_phases_parts128.md).
#ifndef MISLO_PART_BITS
#define MISLO_PART_BITS 10
#endif
constexpr int kPartBits = MISLO_PART_BITS;
constexpr int kParts = 1 << kPartBits;
static_assert(kPartBits >= 6 && kPartBits <= 10, "partition table sizes assume 64..1024 partitions");
constexpr int kPartBlocks = 256;    // max decode/scatter workgroups (per-block partition counts)
constexpr int kMaxDomains = 16;     // posterior columns (10 used, padded to the MFMA tile)
constexpr int kMaxPairs = 48;       // 2-fault hypothesis columns (36 used: pairs of the 9 fault domains)
constexpr int kGroupStripes = 16;   // incident-sum copies (join atomics spread, folded after)
constexpr int kMaxTypes = 128;      // signal_type lookup table size
constexpr uint64_t kEmpty = ~0ull;  // empty top-3 slot
constexpr uint8_t kNoSlot = 0xFF;

// 64-byte event record (collector/records.py EVENT).
struct alignas(64) Event {
  int64_t ts_ns;
  uint64_t value;
  uint64_t trace_h;
  uint32_t pid, tid, pod_id, dst_ip;
  uint16_t signal_type, node_id, svc_id, flags, src_port, dst_port;
  int32_t err;
  uint64_t conn_h;
};
static_assert(sizeof(Event) == 64, "Event must be 64 bytes");

// 32-byte user-space record (collector/records.py USER32; the rocprofiler tool writes it into
// rings created with 32-byte records): fixed-point value, no connection, svc|node from the
// device pod table
struct alignas(32) User32 {
  int64_t ts_ns;
  uint64_t trace_h;
  uint32_t value_milli, pod_id, pid;
  uint8_t signal_type, flags;
  uint16_t node_id;
};
static_assert(sizeof(User32) == 32, "User32 must be 32 bytes");

// 24-byte user-space record (collector/records.py USER24; rings created with 24-byte
// records): USER32 without the unused node id and flags, the timestamp as its low 44 bits
// (decoded to the value nearest the window's newest epoch base: +-2.4 h), pid < 2^22 (pid_max),
// pod id < 2^20 (kPodRows), signal type < 128. 25 % fewer PCIe bytes than USER32.
struct alignas(8) User24 {
  uint64_t trace_h;
  uint32_t value_milli;
  uint32_t ts_lo;    // ts bits 0..31
  uint32_t pid_sig;  // pid (bits 0..21) | signal_type (22..28) | ts_zero (29) | has_gpu (30)
  uint32_t pod_ts;   // pod_id (bits 0..19) | ts bits 32..43 (20..31)
};
static_assert(sizeof(User24) == 24, "User24 must be 24 bytes");
constexpr int kUserTsBits = 44;
__host__ __device__ inline int64_t user24_ts(uint32_t ts_lo, uint32_t pod_ts, uint32_t pid_sig, int64_t base) {
  if (pid_sig & (1u << 29)) return 0;
  const uint64_t t44 = ((uint64_t)(pod_ts >> 20) << 32) | ts_lo;
  const uint64_t mask = (1ull << kUserTsBits) - 1ull;
  const uint64_t d = (t44 - (uint64_t)base) & mask;  // (ts - base) mod 2^44, sign-extended
  const int64_t sd = (int64_t)(d << (64 - kUserTsBits)) >> (64 - kUserTsBits);
  return base + sd;
}

// 16-byte user-space slot (collector/records.py USER16; rings created with 16-byte records):
// User24 without the trace hash, {ts_lo, value_milli, pid_sig, pod_ts}. A record whose pid_sig
// has bit 31 set carries a trace: the next slot is its continuation {trace lo, trace hi,
// kUser16Cont, 0}, a hole (the producers push both in one batch, so no window splits them).
constexpr uint32_t kUser16Cont = 0xFFFFFFFFu;
constexpr uint32_t kUser16Trace = 1u << 31;

// 16-byte wire record (EVENT16 = probes/ebpf/mislo_record.h mislo_event16, the payload of the
// BPF ring's records): timestamp as an offset from one of the window's 4 epoch bases, selected
// by the 2-bit tag in the top of trace_id (ts = base[tag] + ts_off; counts[4..5], [8..13]);
// workload identity as a context id into the device context table {pod, pid, conn32,
// svc<<16|node}; the value in fixed point (1/1000 of the signal's output unit); the kernel's
// trace id (< 2^24, translated to its hash on decode, TraceIds). The probes stamp
// offsets from the epoch the agent last published, so a record written across a window cut
// still decodes exactly.
struct alignas(16) EventC16 {
  uint32_t ts_off, ctx_type, value_milli, trace_id;
};
constexpr int kEpochTagShift = 30;
constexpr uint32_t kTraceIdMask = (1u << kEpochTagShift) - 1u;
constexpr int kCountsLen = 16;  // counts int32[16] (window sizes, epoch bases, context rows)
static_assert(sizeof(EventC16) == 16, "EventC16 must be 16 bytes");
constexpr uint32_t kTsZero = 0xFFFFFFFFu;
// REF packed 40-byte record (ebpf/c/llm_slo_event.h:32-42).
struct __attribute__((packed)) RefEvent {
  uint32_t pid, tid;
  uint64_t timestamp_ns;
  uint32_t signal_type;
  uint64_t value_ns;
  uint16_t conn_src_port, conn_dst_port;
  uint32_t conn_dst_ip;
  int32_t errno_val;
};
static_assert(sizeof(RefEvent) == 40, "RefEvent must be 40 bytes");

// 64-byte span record (collector/records.py SPAN). retr_ms: the request's retrieval time as the
// application reports it (REF's llm.slo.retrieval.{vectordb,network,dns}_ms summed,
// demo/rag-service/main.go:393-397); <= 0 or NaN = no breakdown.
struct alignas(64) Span {
  int64_t ts_ns;
  uint64_t trace_h, conn_h;
  uint32_t pid, pod_id;
  uint16_t node_id, svc_id;
  uint32_t group_id;
  float ttft_ms, latency_ms;
  uint64_t span_h;
  float retr_ms;
  uint32_t flags;  // bit 0 (kSpanLate): the TTFT-SLO deadline passed before the agent's last cut;
                   // bit 1 (kSpanNoSli): SLI counted by the first-token record; bit 2 (kSpanFirstToken):
                   // a first-token record (counted and joined) -- collector/records.py SPAN
};
constexpr uint32_t kSpanLate = 1u, kSpanNoSli = 2u, kSpanFirstToken = 4u;
static_assert(sizeof(Span) == 64, "Span must be 64 bytes");
// 20-byte span record (collector/records.py SPAN20, runtime/csrc/records.h Span20): the fields the
// join reads, with (pod, pid, conn32, svc|node) as a context id into the device context table and
// a trace id. A window uses it when counts[7] == 20 (else 64-byte Span records).
struct __attribute__((packed, aligned(4))) SpanC20 {
  int64_t ts_ns;
  uint32_t trace_id, ctx_id, group_id;
};
static_assert(sizeof(SpanC20) == 20, "SpanC20 must be 20 bytes");

// Decoded signal columns (structure of arrays, one entry per event).
// Row records of the fields the join reads per (signal, key type) visit: one 64-byte line
// per random access instead of one line per column.
struct alignas(64) SigRec {
  int64_t ts;
  uint64_t tr;
  uint64_t cn;
  uint32_t pod, pid, sn;
  float val;
  uint32_t slot;  // kNoSlot = unsupported
  uint32_t pad[5];
};
struct alignas(64) SpanRec {
  int64_t ts;
  uint64_t tr;
  uint64_t cn;
  uint32_t pod, pid, sn, grp;
  uint32_t pad[6];
};
static_assert(sizeof(SigRec) == 64 && sizeof(SpanRec) == 64, "row records are one cache line");

// Per-record partition codes of the 4 join keys (trace, pod+pid, pod+conn, svc+node):
// the key hash's partition (top kPartBits bits) or kNoPart when the key is invalid. The
// signal scatter recomputes full hashes from the row records (into the lists' KeyTs), so only
// 8 bytes per record are stored.
constexpr uint16_t kNoPart = 0xFFFF;
struct alignas(8) PartCodes {
  uint16_t p[4];
};

// One entry of a signal partition list: the row's key hash for the list's key type and its
// timestamp, so the probe streams (hash, ts) in list order and gathers a row record only when
// the key run holds a span within the tier's window.
struct alignas(16) KeyTs {
  uint64_t h;
  int64_t t;
};

// Resident signal generations (the halo). The engine keeps the decoded rows, partition lists and
// list keys of the last kMaxGens windows in place: window k joins the rows of windows k-1.. that
// lie within halo_ms of every later window's latest local record -- the rows a chain of
// per-window halo selections would have carried forward -- without re-copying, re-decoding or
// re-partitioning them (engine.hip k_gen_begin). Generation slots rotate; everything here is
// device state, so a captured window graph replays against whichever slot is current.
constexpr int kMaxGens = 4;  // this window + up to 3 earlier ones (the top-3 key holds the age in 2 bits)
struct GenMeta {
  uint32_t cur;                    // slot of the window being processed
  uint32_t filled;                 // windows held, this one included (<= gens)
  uint32_t n_local[kMaxGens];      // per slot: node-local rows (the other GPUs' rows follow them)
  uint32_t n_rows[kMaxGens];       // per slot: rows
  int64_t tmax_local[kMaxGens];    // per slot: latest local joinable timestamp (the halo anchor; 0 = none)
  uint64_t tlo[kMaxGens], thi[kMaxGens];  // per slot: joinable row time range (order-preserving u64 image)
  int64_t cut[kMaxGens];           // per age: visible rows have ts >= cut (INT64_MAX: none visible)
  uint64_t span_lo, span_hi;       // this window's joinable spans (u64 image)
};
// order-preserving unsigned image of a signed timestamp (atomicMin / atomicMax on u64)
__host__ __device__ inline uint64_t ts_image(int64_t t) { return (uint64_t)t ^ 0x8000000000000000ull; }
__host__ __device__ inline int64_t ts_of_image(uint64_t u) { return (int64_t)(u ^ 0x8000000000000000ull); }

struct SignalCols {
  SigRec* rec;          // [gens][stride] row records
  uint8_t* status;      // this window's rows: 0 ok, 1 warning, 2 error
  PartCodes* part;      // this window's rows
  uint32_t* items = nullptr;  // [gens][kKeyTypes * stride] partition lists (row indices)
  KeyTs* keys = nullptr;      // [gens][kKeyTypes * stride] the lists' (key hash, ts)
  uint32_t* base = nullptr;   // [gens][kKeyTypes * kParts + 1] list offsets
  GenMeta* gen = nullptr;     // nullptr: one generation (slot 0)
  int64_t stride = 0;         // rows per generation
  int gens = 1;
};
constexpr int kBaseLen = kKeyTypes * kParts + 1;  // list offsets per generation
__device__ __forceinline__ uint32_t cur_slot(const SignalCols& c) { return c.gen ? c.gen->cur : 0u; }
__device__ __forceinline__ uint32_t age_slot(const SignalCols& c, uint32_t cur, int age) {
  return (cur + (uint32_t)(c.gens - age)) % (uint32_t)c.gens;
}

struct SpanCols {
  SpanRec* rec;
  PartCodes* part;
};

// Correlation tiers (REF pkg/correlation/dns.go:50-76).
struct JoinParams {
  int64_t outer_ns;       // outer window (default 2 s)
  int64_t win_ns[4];      // effective per-tier window = min(outer, tier window)
  float conf[4];          // 1.0, 0.9, 0.8, 0.65
  float threshold;        // enrichment threshold (default 0.7)
  int fanout;             // max join fanout (3)
  int group_mode;         // incident features: 0 = mean of span top-3 attrs, 1 = mean of all candidates
};

struct Tables {
  int8_t type_slot[kMaxTypes];
  float scale[kSlots];
  float warn[kSlots];
  float err[kSlots];
  float edges[kSlots][kBuckets];  // bucket b holds (edges[b-1], edges[b]]; last edge = +inf
};

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Connection hash of (src_port, dst_port, dst_ip); 0 when no port is set
// (REF builds a conn tuple only when a port != 0, pkg/collector/ringbuf.go:181).
__host__ __device__ inline uint64_t conn_hash(uint32_t sport, uint32_t dport, uint32_t ip) {
  if (sport == 0 && dport == 0) return 0;
  uint64_t packed = ((uint64_t)(sport & 0xFFFF) << 48) | ((uint64_t)(dport & 0xFFFF) << 32) | ip;
  uint64_t h = splitmix64(packed);
  return h ? h : 1;
}

// Key hashes per key type; 0 = invalid key (empty field on this record). The top
// kPartBits bits select the partition.
__host__ __device__ inline uint64_t key_hash(int k, uint64_t trace_h, uint32_t pod, uint32_t pid,
                                             uint64_t conn_h, uint32_t svcnode) {
  uint64_t key;
  switch (k) {
    case 0:
      if (trace_h == 0) return 0;
      key = trace_h ^ 0x1111111111111111ull;
      break;
    case 1:
      if (pod == 0 || pid == 0) return 0;
      key = ((uint64_t)pod << 32 | pid) ^ 0x2222222222222222ull;
      break;
    case 2:
      if (pod == 0 || conn_h == 0) return 0;
      key = splitmix64(conn_h) ^ ((uint64_t)pod * 0x9E3779B97F4A7C15ull) ^ 0x3333333333333333ull;
      break;
    default:
      if ((svcnode >> 16) == 0 || (svcnode & 0xFFFF) == 0) return 0;
      key = (uint64_t)svcnode ^ 0x4444444444444444ull;
      break;
  }
  uint64_t h = splitmix64(key);
  return h ? h : 1;
}

// Fixed-point (1/1000 unit) image of a non-negative value: incident-group sums are exact
// integers, so they are deterministic and all-reduce associatively across GPUs.
__host__ __device__ inline unsigned long long milli_units(float v) {
  const double m = rint((double)v * 1000.0);
  return m > 0.0 ? (unsigned long long)m : 0ull;
}

__host__ __device__ inline int part_of(uint64_t h) { return (int)(h >> (64 - kPartBits)); }

// ---- BPF ring records on the device ---------------------------------------------------------
// The native engine DMAs the BPF ring's bytes as they are: 8-byte header {len | busy | discard,
// pg_off} + a batch of 8 16-byte slots per record (runtime/csrc/bpfring.h), i.e. a 136-byte
// stride; row r of the window is slot r % 8 of record r / 8.
constexpr uint32_t kRbBusy = 1u << 31, kRbDiscard = 1u << 30;
constexpr int kBatchSlots = 8;
constexpr uint32_t kRecPayload = 16 * kBatchSlots;
constexpr int kRecStride = 8 + kRecPayload;
constexpr uint32_t kDefTrace = 0xFD, kDefCtx = 0xFE, kDefFirst = 0xF0;
// the ring bytes of row i's record header and of its slot
__host__ __device__ inline size_t rec_off(int i) { return (size_t)(i >> 3) * kRecStride; }
__host__ __device__ inline size_t slot_off(int i) { return rec_off(i) + 8 + (size_t)(i & 7) * 16; }
// per-window ring accounting (device, packed into the packet): first busy row (min; a batch
// record's first slot), records of another size, context / trace definitions applied, discarded
// records, user-space records
enum RingState { kRsFirstBusy = 0, kRsForeign, kRsDefCtx, kRsDefTrace, kRsDiscard, kRsEvents, kRsOtherShard, kRsLen = 8 };

// the 32-bit connection identity of context rows (runtime/csrc/records.h conn32)
__host__ __device__ inline uint32_t conn32(uint64_t key) {
  return key ? ((uint32_t)(key ^ (key >> 32)) | 1u) : 0u;
}

// Device trace-id table: the kernel's trace id -> the 64-bit trace hash it names (the probes'
// TRACE definitions, applied in ring order before any record that uses the id). Kernel records
// are translated to hashes on decode; user-space records and spans carry hashes already. Every
// row of the join therefore keys on the hash, an identity that is the same on every node, so
// records exchanged between GPUs join without any id translation. Ids wrap at 2^24 (records.h
// kKernelTraceLimit): 128 MiB of HBM, written once per definition, read once per traced event.
struct TraceIds {
  unsigned long long* hash;  // [n], 0 = unknown id
  uint32_t n;
};

__device__ inline uint64_t trace_of(const TraceIds& t, uint32_t id) { return id && id < t.n ? t.hash[id] : 0ull; }

}  // namespace mislo
