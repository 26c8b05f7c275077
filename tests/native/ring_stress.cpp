// Multi-threaded stress of the host ring code under sanitizers (make sanitize-asan /
// sanitize-tsan; tests/test_sanitizers.py). No GPU:
//   1. HostRing (ring.cpp): P producer threads push numbered batches (multi-threaded copies
//      included) while one consumer peeks / releases across wrap-around; every accepted record
//      is seen exactly once and in order per producer, drops are counted, nothing is torn;
//   2. Ringbuf (bpfring.cpp): producer threads reserve / commit / discard / output framed
//      records against the kernel-layout ring while the consumer walks it (busy records stop
//      it, as in libbpf), then a parallel consumer pass and append_framed with threads.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "bpfring.h"
#include "records.h"
#include "ring.h"

using namespace mislo;

#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

struct Rec {  // 64-byte record: producer id, sequence, payload checksum
  uint32_t producer, pad;
  uint64_t seq;
  uint64_t payload[5];
  uint64_t check;
};
static_assert(sizeof(Rec) == 64, "64-byte records");

static uint64_t mix(uint64_t x) { return splitmix64(x); }

static int host_ring(int producers, uint64_t per_producer) {
  const uint64_t cap = 1 << 12;
  std::vector<uint8_t> mem(Ring::bytes_for(cap, 64) + 64);
  void* aligned = reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(mem.data()) + 63) & ~uintptr_t(63));
  Ring* r = Ring::format(aligned, cap, 64);
  std::atomic<int> done{0};
  std::vector<std::thread> ps;
  for (int p = 0; p < producers; ++p)
    ps.emplace_back([&, p] {
      std::vector<Rec> batch(96);
      uint64_t seq = 0;
      while (seq < per_producer) {
        const uint64_t n = std::min<uint64_t>(1 + (mix(seq * 31 + p) % 96), per_producer - seq);
        for (uint64_t i = 0; i < n; ++i) {
          Rec& x = batch[i];
          x.producer = (uint32_t)p;
          x.seq = seq + i;
          for (int q = 0; q < 5; ++q) x.payload[q] = mix((seq + i) * 7 + q + p);
          x.check = x.payload[0] ^ x.payload[4] ^ x.seq;
        }
        // all-or-nothing: a full ring drops the batch; retry it (counted as a drop)
        const int threads = (seq / 96) % 3 == 0 ? 2 : 1;
        if (r->push_batch(batch.data(), n, threads) == n) seq += n;
        else std::this_thread::yield();
      }
      done.fetch_add(1);
    });
  std::vector<uint64_t> next(producers, 0);
  uint64_t seen = 0;
  while (done.load() < producers || r->size()) {
    Segment seg[2];
    const int ns = r->peek(777, seg);
    uint64_t taken = 0;
    for (int s = 0; s < ns; ++s)
      for (uint64_t i = 0; i < seg[s].count; ++i) {
        const Rec* x = reinterpret_cast<const Rec*>(r->records() + (seg[s].index + i) * 64);
        CHECK(x->producer < (uint32_t)producers);
        CHECK(x->seq == next[x->producer]);  // in order, exactly once, per producer
        CHECK(x->check == (x->payload[0] ^ x->payload[4] ^ x->seq));  // not torn
        ++next[x->producer];
        ++taken;
      }
    r->release(taken);
    seen += taken;
    if (!taken) std::this_thread::yield();
  }
  for (auto& t : ps) t.join();
  CHECK(seen == per_producer * producers);
  const unsigned long long dropped = r->header()->dropped.load();
  delete r;  // format() hands out a handle over the caller's memory
  std::printf("host ring: %d producers x %llu records ok (dropped batches %llu)\n", producers,
              (unsigned long long)per_producer, dropped);
  return 0;
}

static int bpf_ring(int producers, int per_producer) {
  const std::string name = "/mislo-stress-" + std::to_string(getpid());
  auto rb = Ringbuf::create_shm(name, 1 << 16);
  std::atomic<int> done{0};
  std::vector<std::thread> ps;
  for (int p = 0; p < producers; ++p)
    ps.emplace_back([&, p] {
      // batch records of kBatchSlots events: per_producer events per producer
      for (int i = 0; i < per_producer; i += (int)kBatchSlots) {
        Rec16 rec[kBatchSlots];
        for (uint32_t j = 0; j < kBatchSlots; ++j)
          rec[j] = Rec16{(uint32_t)(i + (int)j), (uint32_t)(p + 1), (uint32_t)((i + (int)j) * 3), 0};
        const int b = i / (int)kBatchSlots;
        if (b % 3 == 0) {
          while (!rb->output(rec, sizeof(rec))) std::this_thread::yield();
        } else {
          void* s = nullptr;
          while (!(s = rb->reserve(sizeof(rec)))) std::this_thread::yield();
          std::memcpy(s, rec, sizeof(rec));
          rb->commit(s, b % 7 == 0);  // some discarded
        }
      }
      done.fetch_add(1);
    });
  RingbufConsumer cons(rb.get(), 1);
  std::vector<Rec16> out(1 << 14), defs;
  std::vector<int> last(producers, -1);
  uint64_t events = 0, discarded = 0;
  while (done.load() < producers || rb->available()) {
    const ConsumeStats st = cons.consume(out.data(), out.size(), defs);
    for (uint64_t i = 0; i < st.events; ++i) {
      const int p = (int)out[i].ctx_type - 1;
      CHECK(p >= 0 && p < producers);
      CHECK((int)out[i].ts_off > last[p]);  // a producer's records stay in its order
      CHECK(out[i].value_milli == out[i].ts_off * 3);
      last[p] = (int)out[i].ts_off;
    }
    events += st.events;
    discarded += st.discarded * kBatchSlots;
    if (!st.events && !st.discarded) std::this_thread::yield();
  }
  for (auto& t : ps) t.join();
  CHECK(events + discarded == (uint64_t)producers * per_producer);
  // pre-framed appends from a multi-threaded copy, read back by a parallel consumer
  std::vector<Rec16> recs(2000);  // 250 batch records: 34 KiB of a 64 KiB ring
  for (size_t i = 0; i < recs.size(); ++i) recs[i] = Rec16{(uint32_t)i, 9, (uint32_t)i * 3, 0};
  std::vector<uint8_t> img(recs.size() / kBatchSlots * kRecStride);
  frame_records(recs.data(), recs.size(), img.data());
  CHECK(rb->append_framed(img.data(), img.size(), 4));
  RingbufConsumer par(rb.get(), 4);
  const ConsumeStats st = par.consume(out.data(), out.size(), defs);
  CHECK(st.events == recs.size());
  for (size_t i = 0; i < recs.size(); ++i) CHECK(out[i].ts_off == i);
  std::printf("bpf ring: %d producers x %d records ok (%llu discarded)\n", producers, per_producer,
              (unsigned long long)discarded);
  return 0;
}

int main(int argc, char** argv) {
  const int scale = argc > 1 ? std::atoi(argv[1]) : 1;
  if (host_ring(4, 20000 * scale)) return 1;
  if (bpf_ring(4, 20000 * scale)) return 1;
  std::printf("ring stress ok\n");
  return 0;
}
