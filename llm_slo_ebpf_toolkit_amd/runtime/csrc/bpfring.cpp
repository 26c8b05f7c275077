// BPF ring buffer view, kernel-exact emulated producer and the agent's compacting consumer
// (bpfring.h). Reference behaviour: REF pkg/collector/ringbuf.go:120-197 (one Read() per
// record on a goroutine, decoded on the CPU); here a window's records move as one compaction
// into DMA-able memory and are decoded on the GPU (ops/csrc/decode.hip k_decode_wire).
#include "bpfring.h"
#include "ring.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "pool.h"

namespace mislo {

namespace {
constexpr uint64_t kMetaMagic = 0x4d49534c4f524246ull;  // "MISLORBF"
// the kernel's struct bpf_ringbuf keeps its data at page RINGBUF_PGOFF + RINGBUF_POS_PAGES = 3
constexpr uint32_t kDataPgOff = 3;

inline bool pow2(uint64_t x) { return x && !(x & (x - 1)); }

inline uint64_t round8(uint64_t x) { return (x + 7) & ~7ull; }

inline uint32_t load_len(const uint8_t* p) {
  return __atomic_load_n(reinterpret_cast<const uint32_t*>(p), __ATOMIC_ACQUIRE);
}

uint8_t* map_double(int fd, uint64_t page, uint64_t size, bool writable_data) {
  // [meta][consumer][producer][data][data]: reserve the whole range, then map the file over it
  // twice so the data region repeats (a wrapping record reads contiguously)
  const size_t head = 3 * page;
  const size_t total = head + 2 * size;
  void* base = mmap(nullptr, total, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (base == MAP_FAILED) return nullptr;
  uint8_t* b = static_cast<uint8_t*>(base);
  const int prot = PROT_READ | (writable_data ? PROT_WRITE : 0);
  if (mmap(b, head + size, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, fd, 0) == MAP_FAILED ||
      mmap(b + head + size, size, prot, MAP_SHARED | MAP_FIXED, fd, (off_t)head) == MAP_FAILED) {
    munmap(base, total);
    return nullptr;
  }
  return b;
}
}  // namespace

// ---- Ringbuf ----------------------------------------------------------------------------

std::unique_ptr<Ringbuf> Ringbuf::open_map_fd(int fd, uint64_t size) {
  const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
  if (!pow2(size) || size % page) throw std::invalid_argument("ringbuf size must be a power-of-two page multiple");
  std::unique_ptr<Ringbuf> r(new Ringbuf());
  r->page_ = page;
  r->size_ = size;
  void* c = mmap(nullptr, page, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (c == MAP_FAILED) throw std::runtime_error("mmap of the ringbuf consumer page failed");
  r->cons_map_ = static_cast<uint8_t*>(c);
  r->prod_bytes_ = page + 2 * size;
  void* p = mmap(nullptr, r->prod_bytes_, PROT_READ, MAP_SHARED, fd, (off_t)page);
  if (p == MAP_FAILED) {
    munmap(c, page);
    r->cons_map_ = nullptr;
    throw std::runtime_error("mmap of the ringbuf producer/data pages failed");
  }
  r->prod_map_ = static_cast<uint8_t*>(p);
  r->cons_ = reinterpret_cast<uint64_t*>(r->cons_map_);
  r->prod_ = reinterpret_cast<uint64_t*>(r->prod_map_);
  r->data_ = r->prod_map_ + page;
  return r;
}

std::unique_ptr<Ringbuf> Ringbuf::create_shm(const std::string& name, uint64_t size) {
  const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
  if (!pow2(size) || size % page) throw std::invalid_argument("ringbuf size must be a power-of-two page multiple");
  int fd = shm_open(name.c_str(), O_CREAT | O_RDWR | O_TRUNC, 0600);
  if (fd < 0) throw std::runtime_error("shm_open " + name + " failed");
  if (ftruncate(fd, (off_t)(3 * page + size)) != 0 || !mislo_shm_reserve(fd, 3 * page + size)) {
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error("cannot reserve " + std::to_string(3 * page + size) + " bytes of shared memory for " +
                             name + " (/dev/shm too small?)");
  }
  uint8_t* b = map_double(fd, page, size, true);
  if (!b) {
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error("double mapping of " + name + " failed");
  }
  std::unique_ptr<Ringbuf> r(new Ringbuf());
  r->name_ = name;
  r->fd_ = fd;
  r->map_ = b;
  r->map_bytes_ = 3 * page + 2 * size;
  r->page_ = page;
  r->size_ = size;
  r->meta_ = new (b) RbMeta();
  r->meta_->size = size;
  r->meta_->page = page;
  r->meta_->version = 1;
  std::memset(r->meta_->cfg, 0, sizeof(r->meta_->cfg));
  r->meta_->lock.store(0);
  r->meta_->dropped.store(0);
  r->meta_->reserved.store(0);
  r->cons_ = reinterpret_cast<uint64_t*>(b + page);
  r->prod_ = reinterpret_cast<uint64_t*>(b + 2 * page);
  r->data_ = b + 3 * page;
  *r->cons_ = 0;
  *r->prod_ = 0;
  __atomic_store_n(&r->meta_->magic, kMetaMagic, __ATOMIC_RELEASE);
  return r;
}

std::unique_ptr<Ringbuf> Ringbuf::attach_shm(const std::string& name) {
  int fd = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open " + name + " failed (not created?)");
  struct stat st;
  const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
  if (fstat(fd, &st) != 0 || (uint64_t)st.st_size < 4 * page) {
    close(fd);
    throw std::runtime_error(name + ": not an emulated ringbuf");
  }
  const uint64_t size = (uint64_t)st.st_size - 3 * page;
  if (!pow2(size)) {
    close(fd);
    throw std::runtime_error(name + ": bad ringbuf size");
  }
  uint8_t* b = map_double(fd, page, size, true);
  if (!b) {
    close(fd);
    throw std::runtime_error("double mapping of " + name + " failed");
  }
  std::unique_ptr<Ringbuf> r(new Ringbuf());
  r->fd_ = fd;
  r->map_ = b;
  r->map_bytes_ = 3 * page + 2 * size;
  r->page_ = page;
  r->size_ = size;
  r->meta_ = reinterpret_cast<RbMeta*>(b);
  if (__atomic_load_n(&r->meta_->magic, __ATOMIC_ACQUIRE) != kMetaMagic || r->meta_->size != size)
    throw std::runtime_error(name + ": ringbuf meta page mismatch");
  r->cons_ = reinterpret_cast<uint64_t*>(b + page);
  r->prod_ = reinterpret_cast<uint64_t*>(b + 2 * page);
  r->data_ = b + 3 * page;
  return r;
}

Ringbuf::~Ringbuf() {
  if (map_) munmap(map_, map_bytes_);
  if (cons_map_) munmap(cons_map_, page_);
  if (prod_map_) munmap(prod_map_, prod_bytes_);
  if (fd_ >= 0) close(fd_);
  if (!name_.empty()) shm_unlink(name_.c_str());
}

uint32_t Ringbuf::pg_off_of(uint64_t pos) const {
  return kDataPgOff + (uint32_t)((pos & mask()) / page_);
}

void Ringbuf::lock() {
  auto& l = meta_->lock;
  for (;;) {
    if (l.exchange(1, std::memory_order_acquire) == 0) return;
    while (l.load(std::memory_order_relaxed)) std::this_thread::yield();
  }
}

void Ringbuf::unlock() { meta_->lock.store(0, std::memory_order_release); }

void* Ringbuf::reserve(uint32_t size) {
  if (!meta_) throw std::logic_error("reserve: the producer side of a real ringbuf is the kernel's");
  if (size > (size_ >> 3) || size == 0) return nullptr;  // RINGBUF_MAX_RECORD_SZ-style bound
  const uint64_t len = round8((uint64_t)size + kRbHdrSz);
  const uint64_t cons = consumer_pos();
  lock();
  const uint64_t prod = *prod_;
  const uint64_t next = prod + len;
  if (next - cons > mask()) {  // would overrun unconsumed data
    unlock();
    meta_->dropped.fetch_add(1, std::memory_order_relaxed);
    return nullptr;
  }
  uint8_t* hdr = data_ + (prod & mask());
  RbHeader* h = reinterpret_cast<RbHeader*>(hdr);
  h->pg_off = pg_off_of(prod);
  __atomic_store_n(&h->len, size | kRbBusyBit, __ATOMIC_RELAXED);
  __atomic_store_n(prod_, next, __ATOMIC_RELEASE);
  unlock();
  meta_->reserved.fetch_add(1, std::memory_order_relaxed);
  return hdr + kRbHdrSz;
}

void Ringbuf::commit(void* sample, bool discard) {
  uint32_t* len = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(sample) - kRbHdrSz);
  uint32_t v = __atomic_load_n(len, __ATOMIC_RELAXED) ^ kRbBusyBit;
  if (discard) v |= kRbDiscardBit;
  __atomic_exchange_n(len, v, __ATOMIC_ACQ_REL);
}

bool Ringbuf::output(const void* payload, uint32_t size) {
  void* p = reserve(size);
  if (!p) return false;
  std::memcpy(p, payload, size);
  commit(p, false);
  return true;
}

bool Ringbuf::append_framed(const uint8_t* bytes, uint64_t n, int threads) {
  if (!meta_) throw std::logic_error("append_framed: emulated rings only");
  if (n % 8) throw std::invalid_argument("framed image must be a multiple of 8 bytes");
  if (n == 0) return true;
  const uint64_t cons = consumer_pos();
  lock();
  const uint64_t prod = *prod_;
  if (prod + n - cons > mask()) {
    unlock();
    return false;
  }
  // copy (the double mapping takes care of the wrap), then fix the page offsets of the
  // headers for their new positions and publish everything with one release store
  const uint64_t at = prod & mask();
  const uint64_t first = std::min<uint64_t>(n, size_ - at);
  parallel_memcpy(data_ + at, bytes, first, threads);
  if (first < n) parallel_memcpy(data_, bytes + first, n - first, threads);
  for (uint64_t off = 0; off < n;) {
    RbHeader* h = reinterpret_cast<RbHeader*>(data_ + ((prod + off) & mask()));
    h->pg_off = pg_off_of(prod + off);
    const uint32_t len = h->len & ~(kRbBusyBit | kRbDiscardBit);
    off += round8((uint64_t)len + kRbHdrSz);
  }
  __atomic_store_n(prod_, prod + n, __ATOMIC_RELEASE);
  unlock();
  return true;
}

void frame_records(const Rec16* recs, uint64_t n, uint8_t* out) {
  if (n % kBatchSlots) throw std::invalid_argument("frame_records: whole batches of 8 slots only");
  for (uint64_t i = 0; i < n / kBatchSlots; ++i) {
    RbHeader h{kRecPayload, 0};
    std::memcpy(out + i * kRecStride, &h, sizeof(h));
    std::memcpy(out + i * kRecStride + kRbHdrSz, &recs[i * kBatchSlots], kRecPayload);
  }
}

namespace {
// One batch record's slots: events to `out` (while there is room; returns false when full),
// definitions to `defs`, pads counted.
template <class Def>
bool take_slots(const uint8_t* payload, Rec16* out, uint64_t cap, uint64_t* k, Def&& def, uint64_t* pads) {
  Rec16 r[kBatchSlots];
  std::memcpy(r, payload, sizeof(r));
  uint64_t ev = 0;
  for (uint32_t j = 0; j < kBatchSlots; ++j) ev += (r[j].ctx_type & 0xFFu) < kDefFirst;
  if (*k + ev > cap) return false;  // the whole batch waits for the next window
  for (uint32_t j = 0; j < kBatchSlots; ++j) {
    const uint32_t t = r[j].ctx_type & 0xFFu;
    if (t < kDefFirst)
      out[(*k)++] = r[j];
    else if (t == kPad)
      ++*pads;
    else
      def(r[j]);
  }
  return true;
}
}  // namespace

// ---- RingbufConsumer --------------------------------------------------------------------

RingbufConsumer::RingbufConsumer(Ringbuf* rb, int threads) : rb_(rb) {
  if (!rb) throw std::invalid_argument("null ringbuf");
  pool_ = std::make_unique<WorkerPool>(std::max(1, std::min(threads, 64)));
}

RingbufConsumer::~RingbufConsumer() = default;

int RingbufConsumer::threads() const { return pool_->threads(); }

// libbpf ringbuf_process_ring semantics, one record at a time: the reference walk for any
// record size (other programs sharing the map, a partially filled tail).
ConsumeStats RingbufConsumer::consume_serial(Rec16* out, uint64_t cap, std::vector<Rec16>& defs, uint64_t cons,
                                             uint64_t prod) {
  ConsumeStats st;
  st.serial = true;
  st.begin_pos = cons;
  const uint8_t* data = rb_->data();
  const uint64_t mask = rb_->mask();
  while (cons < prod) {
    const uint8_t* hdr = data + (cons & mask);
    const uint32_t len = load_len(hdr);
    if (len & kRbBusyBit) {
      st.busy_stop = true;
      break;
    }
    const uint32_t plen = len & ~(kRbBusyBit | kRbDiscardBit);
    if (!(len & kRbDiscardBit) && plen == kRecPayload) {
      // window full: the record stays for the next window
      if (!take_slots(hdr + kRbHdrSz, out, cap, &st.events, [&](const Rec16& d) { defs.push_back(d), ++st.defs; },
                      &st.pads))
        break;
    } else if (len & kRbDiscardBit) {
      ++st.discarded;
    } else {
      ++st.foreign;
    }
    cons += round8((uint64_t)plen + kRbHdrSz);
  }
  st.end_pos = cons;
  rb_->set_consumer_pos(cons);
  return st;
}

ConsumeStats RingbufConsumer::consume(Rec16* out, uint64_t cap, std::vector<Rec16>& defs, uint64_t limit) {
  const uint64_t cons = rb_->consumer_pos();
  uint64_t prod = rb_->producer_pos();
  if (limit < prod && limit >= cons) prod = limit;
  if (prod <= cons) {
    ConsumeStats st;
    st.begin_pos = st.end_pos = cons;
    return st;
  }
  const uint64_t span = prod - cons;
  // fast path: every record in range is a batch (136 ring bytes), so record i sits at
  // cons + 136 i and chunks can be compacted independently; a foreign size anywhere sends the
  // window down the serial walk
  if (span % kRecStride) return consume_serial(out, cap, defs, cons, prod);
  const uint64_t n = span / kRecStride;
  // defs / pads / discards only shrink the output: scanning cap / 8 batches always fits
  const uint64_t n_scan = std::min<uint64_t>(n, cap / kBatchSlots);
  const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)threads() * 2, n_scan / 8192 + 1));
  if ((int)tasks_.size() < nt) tasks_.resize(nt);
  const uint8_t* data = rb_->data();
  const uint64_t mask = rb_->mask();
  pool_->run(nt, [&](int t) {
    Task& tk = tasks_[t];
    tk.lo = n_scan * t / nt;
    tk.hi = n_scan * (t + 1) / nt;
    tk.k = tk.discards = tk.pads = 0;
    tk.busy = -1;
    tk.foreign = false;
    tk.defs.clear();
    Rec16* dst = out + tk.lo * kBatchSlots;
    for (uint64_t i = tk.lo; i < tk.hi; ++i) {
      const uint8_t* hdr = data + ((cons + i * kRecStride) & mask);
      const uint32_t len = load_len(hdr);
      if (len & kRbBusyBit) {
        tk.busy = (int64_t)i;
        return;
      }
      if ((len & ~(kRbBusyBit | kRbDiscardBit)) != kRecPayload) {
        tk.foreign = true;
        return;
      }
      if (len & kRbDiscardBit) {
        ++tk.discards;
        continue;
      }
      take_slots(hdr + kRbHdrSz, dst, ~0ull, &tk.k, [&](const Rec16& d) { tk.defs.emplace_back(i, d); }, &tk.pads);
    }
  });
  for (int t = 0; t < nt; ++t)
    if (tasks_[t].foreign) return consume_serial(out, cap, defs, cons, prod);
  ConsumeStats st;
  st.begin_pos = cons;
  uint64_t end = n_scan;  // records consumed: up to the first busy one
  int last = nt - 1;
  for (int t = 0; t < nt; ++t)
    if (tasks_[t].busy >= 0) {
      end = (uint64_t)tasks_[t].busy;
      last = t;
      st.busy_stop = true;
      break;
    }
  // close the gaps left by definitions / discards (rare after start-up): chunk t's records
  // move from out + lo_t down to the running total
  uint64_t w = 0;
  for (int t = 0; t <= last; ++t) {
    Task& tk = tasks_[t];
    if (w != tk.lo * kBatchSlots && tk.k) std::memmove(out + w, out + tk.lo * kBatchSlots, tk.k * sizeof(Rec16));
    w += tk.k;
    st.discarded += tk.discards;
    st.pads += tk.pads;
    for (auto& d : tk.defs) defs.push_back(d.second);
    st.defs += tk.defs.size();
  }
  st.events = w;
  st.end_pos = cons + end * kRecStride;
  rb_->set_consumer_pos(st.end_pos);
  return st;
}

}  // namespace mislo
