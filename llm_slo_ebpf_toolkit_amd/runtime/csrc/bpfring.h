// The kernel -> agent hand-off: a BPF ring buffer map (BPF_MAP_TYPE_RINGBUF, the probes'
// `mislo_events`) read the way the kernel lays it out for user space (kernel/bpf/ringbuf.c):
//
//   mmap offset 0          : one page, consumer_pos (u64), read-write for the consumer
//   mmap offset PAGE       : one page, producer_pos (u64), read-only
//   mmap offset 2 * PAGE   : the data pages, mapped TWICE back to back (read-only), so a record
//                            that wraps past the end is still contiguous in the mapping
//
// Each record is an 8-byte header {u32 len; u32 pg_off} followed by `len` payload bytes, the
// whole rounded up to 8 bytes. The kernel reserves under a spinlock, writes the header with
// BPF_RINGBUF_BUSY_BIT, publishes producer_pos (release), copies the payload and commits by
// xchg'ing the header (busy bit cleared, BPF_RINGBUF_DISCARD_BIT set on discard). A consumer
// may only pass records whose header is not busy, and frees space by storing consumer_pos.
//
// The agent's consumer (RingbufConsumer) does not hand records to a callback one by one, as
// libbpf's ring_buffer__consume does: it compacts a window's committed EVENT16 slots
// (probes/ebpf/mislo_record.h mislo_event16; batches of 8 per 136-byte record) straight into the
// pinned buffer the window is DMA'd from, on a worker pool, diverting the probes' id
// definition slots (mislo_def16: context rows, trace ids) to a side list, skipping pads and
// discarded records and stopping at the first busy one (libbpf semantics: nothing past it is
// consumed).
//
// For tests, the benchmark and the CPU-only CI, `Ringbuf::create_shm` builds the identical
// user-visible layout over shared memory (double-mapped data, a meta page holding the
// emulated `mislo_cfg` array), and `reserve` / `commit` / `output` reproduce the kernel
// producer exactly (same spinlock-serialised reservation order, header bits, pg_off, 8-byte
// rounding, overflow check against consumer_pos), so the consumer runs unchanged on both.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace mislo {

class WorkerPool;

constexpr uint32_t kRbBusyBit = 1u << 31;
constexpr uint32_t kRbDiscardBit = 1u << 30;
constexpr uint32_t kRbHdrSz = 8;
// A ring record is a batch: the probes stage 16-byte slots per CPU (mislo_probe.h mislo_stage)
// and put kBatchSlots of them on the ring in one record, so the 8-byte header is paid once per
// batch instead of once per event (17 ring bytes per event instead of 24). Row r of a window is
// slot r % kBatchSlots of record r / kBatchSlots.
constexpr uint32_t kSlotBytes = 16;                      // mislo_event16 / mislo_def16 / pad
constexpr uint32_t kBatchSlots = 8;
constexpr uint32_t kRecPayload = kSlotBytes * kBatchSlots;  // 128
constexpr uint32_t kRecStride = kRbHdrSz + kRecPayload;     // 136 ring bytes per record
constexpr int kCfgSlots = 128;                              // mislo_cfg entries (u64)

// non-event slots (mislo_record.h): low byte of ctx_type
constexpr uint32_t kDefTrace = 0xFD;  // {ts_off = trace id, ctx_type, value_milli = hash lo, trace_tag = hash hi}
constexpr uint32_t kDefCtx = 0xFE;    // {ts_off = conn32, ctx_type = type | id << 8, value_milli = pod, trace_tag = pid}
constexpr uint32_t kPad = 0xFC;       // an unused slot of a batch flushed before it filled
constexpr uint32_t kDefFirst = 0xF0;  // types >= this never reach the GPU as events

struct Rec16 {
  uint32_t ts_off, ctx_type, value_milli, trace_tag;
};
static_assert(sizeof(Rec16) == 16, "EVENT16 is 16 bytes");

struct RbHeader {
  uint32_t len;
  uint32_t pg_off;
};

// Emulated-map meta page (shared memory only; page 0 of the shm file).
struct alignas(64) RbMeta {
  uint64_t magic;
  uint64_t size;     // data bytes (power of two, multiple of the page size)
  uint64_t page;
  uint64_t version;
  alignas(64) uint64_t cfg[kCfgSlots];  // emulated mislo_cfg (BPF array map)
  alignas(64) std::atomic<uint32_t> lock;  // the kernel's rb->spinlock
  std::atomic<uint64_t> dropped;           // failed reservations (ring full)
  std::atomic<uint64_t> reserved;          // successful reservations
};

class Ringbuf {
 public:
  // A real BPF ringbuf map (fd from BPF_OBJ_GET of the pinned map), `size` = max_entries.
  static std::unique_ptr<Ringbuf> open_map_fd(int fd, uint64_t size);
  // Emulated ring in POSIX shared memory `name` (created / attached).
  static std::unique_ptr<Ringbuf> create_shm(const std::string& name, uint64_t size);
  static std::unique_ptr<Ringbuf> attach_shm(const std::string& name);
  ~Ringbuf();
  Ringbuf(const Ringbuf&) = delete;
  Ringbuf& operator=(const Ringbuf&) = delete;

  uint64_t size() const { return size_; }
  uint64_t mask() const { return size_ - 1; }
  uint64_t page() const { return page_; }
  const uint8_t* data() const { return data_; }
  bool emulated() const { return meta_ != nullptr; }
  RbMeta* meta() const { return meta_; }
  uint64_t* cfg() const { return meta_ ? meta_->cfg : nullptr; }

  uint64_t consumer_pos() const { return __atomic_load_n(cons_, __ATOMIC_ACQUIRE); }
  uint64_t producer_pos() const { return __atomic_load_n(prod_, __ATOMIC_ACQUIRE); }
  void set_consumer_pos(uint64_t p) { __atomic_store_n(cons_, p, __ATOMIC_RELEASE); }
  uint64_t available() const { return producer_pos() - consumer_pos(); }

  // ---- emulated producer (kernel __bpf_ringbuf_reserve / bpf_ringbuf_commit) ------------
  // Returns the payload pointer (busy record) or nullptr when the ring is full (counted).
  void* reserve(uint32_t size);
  void commit(void* sample, bool discard);
  bool output(const void* payload, uint32_t size);  // bpf_ringbuf_output
  // Appends pre-framed, committed records (a byte image of headers + payloads whose pg_off
  // fields are rewritten for their new position) under the producer lock and publishes them
  // with one producer_pos store. Fails (nothing written) when they do not fit.
  bool append_framed(const uint8_t* bytes, uint64_t n, int threads = 1);
  std::string name() const { return name_; }

 private:
  Ringbuf() = default;
  uint32_t pg_off_of(uint64_t pos) const;
  void lock();
  void unlock();
  std::string name_;
  int fd_ = -1;
  uint8_t* map_ = nullptr;   // emulated: the whole reserved range
  size_t map_bytes_ = 0;
  uint8_t* cons_map_ = nullptr;  // real map: the two separate mappings
  uint8_t* prod_map_ = nullptr;
  size_t prod_bytes_ = 0;
  RbMeta* meta_ = nullptr;
  uint64_t* cons_ = nullptr;
  uint64_t* prod_ = nullptr;
  uint8_t* data_ = nullptr;
  uint64_t size_ = 0, page_ = 4096;
};

struct ConsumeStats {
  uint64_t events = 0;     // EVENT16 slots written to the output
  uint64_t defs = 0;       // definition slots diverted
  uint64_t pads = 0;       // unused slots of partial batches
  uint64_t discarded = 0;  // records committed with the discard bit
  uint64_t foreign = 0;    // records of another payload size (skipped, counted)
  uint64_t begin_pos = 0, end_pos = 0;  // consumed ring range [begin, end)
  bool busy_stop = false;  // stopped at a record still being written
  bool serial = false;     // took the generic (variable-size) walk
};

class RingbufConsumer {
 public:
  RingbufConsumer(Ringbuf* rb, int threads);
  ~RingbufConsumer();
  // Consume committed records in [consumer_pos, min(limit, producer_pos)) into `out`
  // (EVENT16, at most `cap` records), definitions appended to `defs`; frees the consumed
  // space (consumer_pos store-release) before returning.
  ConsumeStats consume(Rec16* out, uint64_t cap, std::vector<Rec16>& defs, uint64_t limit = ~0ull);
  Ringbuf* ring() const { return rb_; }
  int threads() const;

 private:
  ConsumeStats consume_serial(Rec16* out, uint64_t cap, std::vector<Rec16>& defs, uint64_t cons, uint64_t prod);
  Ringbuf* rb_;
  std::unique_ptr<WorkerPool> pool_;
  struct Task {
    uint64_t lo, hi, k, discards, pads;
    int64_t busy;  // first busy index or -1
    bool foreign;
    std::vector<std::pair<uint64_t, Rec16>> defs;
  };
  std::vector<Task> tasks_;
};

// Frames batches of kBatchSlots slots as committed ring records (header + 128-byte payload,
// pg_off left 0): the byte image Ringbuf::append_framed publishes. `n` is a multiple of kBatchSlots.
void frame_records(const Rec16* recs, uint64_t n, uint8_t* out);

inline Rec16 pad_slot() { return Rec16{0, kPad, 0, 0}; }

}  // namespace mislo
