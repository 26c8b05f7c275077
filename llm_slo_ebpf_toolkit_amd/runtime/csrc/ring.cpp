#include "ring.h"

#include "pool.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include <cstring>
#include <new>
#include <string>
#include <thread>

namespace mislo {

static inline bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }

size_t Ring::bytes_for(uint64_t capacity, uint32_t rec_size) {
  return kRingHeaderBytes + (size_t)capacity * rec_size;
}

Ring* Ring::format(void* mem, uint64_t capacity, uint32_t rec_size) {
  if (!mem || !is_pow2(capacity) || rec_size == 0 || ((uintptr_t)mem & 63)) return nullptr;
  static_assert(sizeof(RingHeader) <= kRingHeaderBytes, "header too large");
  auto* h = new (mem) RingHeader();
  h->capacity = capacity;
  h->rec_size = rec_size;
  h->version = 1;
  h->total_bytes = bytes_for(capacity, rec_size);
  h->head.store(0, std::memory_order_relaxed);
  h->tail.store(0, std::memory_order_relaxed);
  h->lock.store(0, std::memory_order_relaxed);
  h->pushed.store(0, std::memory_order_relaxed);
  h->dropped.store(0, std::memory_order_relaxed);
  h->high_water.store(0, std::memory_order_relaxed);
  h->batches.store(0, std::memory_order_relaxed);
  h->stolen.store(0, std::memory_order_relaxed);
  h->drop_mask.store(0, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  h->magic = kRingMagic;
  return attach(mem);
}

Ring* Ring::attach(void* mem) {
  auto* h = reinterpret_cast<RingHeader*>(mem);
  if (!h || h->magic != kRingMagic) return nullptr;
  Ring* r = new Ring();
  r->hdr_ = h;
  r->recs_ = reinterpret_cast<uint8_t*>(mem) + kRingHeaderBytes;
  return r;
}

uint64_t Ring::push_batch(const void* recs, uint64_t n, int threads) {
  if (n == 0) return 0;
  RingHeader* h = hdr_;
  const uint64_t cap = h->capacity;
  // producer lock: holds the owner's pid, so a producer process that died holding it (the
  // ring lives in shared memory) is detected and the lock taken over. Safe because the
  // release store of `head` is the commit point: a dead owner either published its batch
  // or left `head` where it was (its partial copy is overwritten).
  const uint32_t me = (uint32_t)getpid();
  for (uint32_t spins = 0;;) {
    uint32_t cur = 0;
    if (h->lock.compare_exchange_weak(cur, me, std::memory_order_acquire, std::memory_order_relaxed)) break;
    if (cur != 0 && cur != me && ++spins >= 4096) {
      spins = 0;
      if (kill((pid_t)cur, 0) != 0 && errno == ESRCH &&
          h->lock.compare_exchange_strong(cur, me, std::memory_order_acquire, std::memory_order_relaxed)) {
        h->stolen.fetch_add(1, std::memory_order_relaxed);
        break;
      }
    }
    std::this_thread::yield();
  }
  const uint64_t head = h->head.load(std::memory_order_relaxed);
  const uint64_t tail = h->tail.load(std::memory_order_acquire);
  if (head - tail + n > cap) {
    h->lock.store(0, std::memory_order_release);
    h->dropped.fetch_add(n, std::memory_order_relaxed);
    return 0;
  }
  const uint32_t rs = h->rec_size;
  const uint64_t idx = head & (cap - 1);
  const uint64_t first = (idx + n <= cap) ? n : cap - idx;
  parallel_memcpy(recs_ + idx * rs, recs, first * rs, threads);
  if (first < n) parallel_memcpy(recs_, reinterpret_cast<const uint8_t*>(recs) + first * rs, (n - first) * rs, threads);
  h->head.store(head + n, std::memory_order_release);
  h->lock.store(0, std::memory_order_release);
  h->pushed.fetch_add(n, std::memory_order_relaxed);
  h->batches.fetch_add(1, std::memory_order_relaxed);
  const uint64_t fill = head + n - tail;
  uint64_t hw = h->high_water.load(std::memory_order_relaxed);
  while (fill > hw && !h->high_water.compare_exchange_weak(hw, fill, std::memory_order_relaxed)) {
  }
  return n;
}

int Ring::peek(uint64_t max_records, Segment out[2]) const {
  const uint64_t head = hdr_->head.load(std::memory_order_acquire);
  const uint64_t tail = hdr_->tail.load(std::memory_order_relaxed);
  uint64_t avail = head - tail;
  if (avail > max_records) avail = max_records;
  if (avail == 0) return 0;
  const uint64_t cap = hdr_->capacity;
  const uint64_t idx = tail & (cap - 1);
  const uint64_t first = (idx + avail <= cap) ? avail : cap - idx;
  out[0] = Segment{tail, idx, first};
  if (first == avail) return 1;
  out[1] = Segment{tail + first, 0, avail - first};
  return 2;
}

void Ring::release(uint64_t n) {
  const uint64_t tail = hdr_->tail.load(std::memory_order_relaxed);
  const uint64_t head = hdr_->head.load(std::memory_order_acquire);
  if (n > head - tail) n = head - tail;
  hdr_->tail.store(tail + n, std::memory_order_release);
}

uint64_t Ring::size() const {
  return hdr_->head.load(std::memory_order_acquire) - hdr_->tail.load(std::memory_order_acquire);
}

}  // namespace mislo

using mislo::Ring;

namespace {
struct ShmRing {
  Ring* ring;
  void* base;
  size_t bytes;
};
}  // namespace

extern "C" {

bool mislo_shm_reserve(int fd, size_t bytes) {
  // a capacity check, not an allocation: the pages stay unallocated so that the first process
  // to touch them -- the producer, bound to its GPU's NUMA node -- places them (first touch)
  struct statvfs sv;
  if (fstatvfs(fd, &sv) != 0) return true;  // cannot tell: as before
  return (unsigned long long)sv.f_bavail * sv.f_frsize >= bytes;
}

void* mislo_ring_create_shm(const char* name, uint64_t capacity, uint32_t rec_size) {
  const size_t bytes = Ring::bytes_for(capacity, rec_size);
  int fd = shm_open(name, O_CREAT | O_RDWR | O_TRUNC, 0600);
  if (fd < 0) return nullptr;
  // a tmpfs (/dev/shm) too small for a sparse ftruncate'd ring fails here, instead of SIGBUS-ing
  // the first producer that touches a page it cannot back
  if (ftruncate(fd, (off_t)bytes) != 0 || !mislo_shm_reserve(fd, bytes)) {
    close(fd);
    shm_unlink(name);
    return nullptr;
  }
  void* base = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base == MAP_FAILED) return nullptr;
  Ring* r = Ring::format(base, capacity, rec_size);
  if (!r) {
    munmap(base, bytes);
    return nullptr;
  }
  return new ShmRing{r, base, bytes};
}

void* mislo_ring_open_shm(const char* name) {
  int fd = shm_open(name, O_RDWR, 0600);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < (off_t)mislo::kRingHeaderBytes) {
    close(fd);
    return nullptr;
  }
  void* base = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base == MAP_FAILED) return nullptr;
  Ring* r = Ring::attach(base);
  if (!r) {
    munmap(base, (size_t)st.st_size);
    return nullptr;
  }
  return new ShmRing{r, base, (size_t)st.st_size};
}

void mislo_ring_close(void* ring) {
  auto* s = reinterpret_cast<ShmRing*>(ring);
  if (!s) return;
  munmap(s->base, s->bytes);
  delete s->ring;
  delete s;
}

int mislo_ring_unlink_shm(const char* name) { return shm_unlink(name); }

int mislo_ring_push(void* ring, const void* rec) {
  return reinterpret_cast<ShmRing*>(ring)->ring->push(rec) ? 1 : 0;
}

uint64_t mislo_ring_push_batch(void* ring, const void* recs, uint64_t n) {
  return reinterpret_cast<ShmRing*>(ring)->ring->push_batch(recs, n);
}

void* mislo_ring_handle_ring(void* ring) { return ring ? reinterpret_cast<ShmRing*>(ring)->ring : nullptr; }

uint64_t mislo_ring_size(void* ring) { return reinterpret_cast<ShmRing*>(ring)->ring->size(); }

uint32_t mislo_ring_rec_size(void* ring) { return reinterpret_cast<ShmRing*>(ring)->ring->rec_size(); }

uint64_t mislo_ring_dropped(void* ring) {
  return reinterpret_cast<ShmRing*>(ring)->ring->header()->dropped.load(std::memory_order_relaxed);
}
uint32_t mislo_ring_drop_mask(void* ring) {
  return reinterpret_cast<ShmRing*>(ring)->ring->header()->drop_mask.load(std::memory_order_relaxed);
}
void mislo_ring_set_drop_mask(void* ring, uint32_t mask) {
  reinterpret_cast<ShmRing*>(ring)->ring->header()->drop_mask.store(mask, std::memory_order_relaxed);
}
}
