// Bounded MPSC ring of fixed-size event records in (optionally shared, optionally pinned)
// host memory -- the hand-off between probe producers (BPF ring-buffer readers, the
// rocprofiler-sdk tool library inside GPU workloads, replay threads) and the agent's
// window consumer, which DMAs contiguous record ranges straight into the per-GPU HBM
// event store.
//
// Design (chosen so the consumer's per-window CPU cost is O(1), not O(records)):
//   * producers serialise on a tiny lock word holding the owner's pid (uncontended in the
//     intended deployment of one ring per producer source; a lock left by a producer process
//     that died is taken over), copy records in, and publish with a single release store of
//     `head`; a full ring DROPS the batch and counts it (bpf_ringbuf_reserve semantics) --
//     producers never block;
//   * the single consumer reads `head` (acquire), hands out at most two contiguous
//     segments (wrap-around) for DMA, and release()s them after the copy completed.
// head/tail are monotonic 64-bit counters; capacity is a power of two.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>

namespace mislo {

struct alignas(64) RingHeader {
  uint64_t magic;
  uint64_t capacity;     // records, power of two
  uint32_t rec_size;     // bytes per record (64 for EVENT/SPAN, 40 for REF)
  uint32_t version;
  uint64_t total_bytes;  // header + records
  alignas(64) std::atomic<uint64_t> head;     // producer publish position
  alignas(64) std::atomic<uint64_t> tail;     // consumer release position
  alignas(64) std::atomic<uint32_t> lock;     // producer lock: owner pid, 0 = free
  std::atomic<uint64_t> pushed;
  std::atomic<uint64_t> dropped;
  std::atomic<uint64_t> high_water;
  std::atomic<uint64_t> batches;
  std::atomic<uint64_t> stolen;  // locks taken over from dead producers
  // Shedding control (agent -> producers): bit t set = producers stop emitting signal type t
  // (t < 32). The agent's overhead guard sets it before it detaches probes; producers that
  // attach (the rocprofiler tool inside workloads) read it per record.
  alignas(64) std::atomic<uint32_t> drop_mask;
};

constexpr uint64_t kRingMagic = 0x4d49534c4f52494eull;  // "MISLORIN"
constexpr size_t kRingHeaderBytes = 512;

struct Segment {
  uint64_t pos;    // absolute position of the first record
  uint64_t index;  // slot index in the record array
  uint64_t count;
};

class Ring {
 public:
  static size_t bytes_for(uint64_t capacity, uint32_t rec_size);
  // Lay out a ring inside caller memory (64-byte aligned, bytes_for() bytes).
  static Ring* format(void* mem, uint64_t capacity, uint32_t rec_size);
  // Attach to an already formatted region (e.g. a shared-memory mapping).
  static Ring* attach(void* mem);

  bool push(const void* rec) { return push_batch(rec, 1) == 1; }
  // all-or-nothing; returns accepted count (large batches copy on `threads` threads)
  uint64_t push_batch(const void* recs, uint64_t n, int threads = 1);

  int peek(uint64_t max_records, Segment out[2]) const;  // consumer: 0..2 segments
  void release(uint64_t n);                               // consumer

  uint8_t* records() const { return recs_; }
  RingHeader* header() const { return hdr_; }
  uint64_t capacity() const { return hdr_->capacity; }
  uint32_t rec_size() const { return hdr_->rec_size; }
  uint64_t size() const;

 private:
  RingHeader* hdr_ = nullptr;
  uint8_t* recs_ = nullptr;
};

}  // namespace mislo

extern "C" {
// C ABI for external producers (BPF loader, rocprofiler-sdk tool library) and tests.
// Whether a shared-memory file's filesystem has room for `bytes` (false: a tmpfs too small).
bool mislo_shm_reserve(int fd, size_t bytes);
void* mislo_ring_create_shm(const char* name, uint64_t capacity, uint32_t rec_size);
void* mislo_ring_open_shm(const char* name);
void mislo_ring_close(void* ring);
int mislo_ring_unlink_shm(const char* name);
int mislo_ring_push(void* ring, const void* rec);
uint64_t mislo_ring_push_batch(void* ring, const void* recs, uint64_t n);
uint64_t mislo_ring_size(void* ring);
uint32_t mislo_ring_rec_size(void* ring);  // 64 (EVENT) or 32 (USER32)
// The mislo::Ring* behind a handle from mislo_ring_create_shm / mislo_ring_open_shm.
void* mislo_ring_handle_ring(void* ring);
uint64_t mislo_ring_dropped(void* ring);
// The ring's shedding mask (bit t: drop signal type t) -- read by producers, set by the agent.
uint32_t mislo_ring_drop_mask(void* ring);
void mislo_ring_set_drop_mask(void* ring, uint32_t mask);
}
