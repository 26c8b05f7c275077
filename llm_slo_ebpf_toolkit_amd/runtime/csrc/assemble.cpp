#include "assemble.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>

namespace mislo {

WindowAssembler::WindowAssembler(const SlotLayout& L, AgentTables* tables, RingbufConsumer* kernel, Ring* user_events,
                                 Ring* spans)
    : L_(L), tables_(tables), kernel_(kernel), user_(user_events), spans_(spans) {
  if (!tables) throw std::invalid_argument("WindowAssembler needs AgentTables");
  if (user_events && user_events->rec_size() != sizeof(EventRec))
    throw std::invalid_argument("user event ring must hold 64-byte EVENT records");
  if (spans && spans->rec_size() != sizeof(SpanRec64)) throw std::invalid_argument("span ring must hold 64-byte SPAN records");
}

namespace {
// up to `max` records of `ring` at or before position `limit`, as <= 2 contiguous segments
int ring_take(Ring* ring, uint64_t limit, uint64_t max, Segment seg[2]) {
  const uint64_t tail = ring->header()->tail.load(std::memory_order_relaxed);
  uint64_t n = max;
  if (limit != ~0ull) n = std::min<uint64_t>(n, limit > tail ? limit - tail : 0);
  return n ? ring->peek(n, seg) : 0;
}
}  // namespace

AssembleResult WindowAssembler::assemble(uint8_t* slot, const int64_t bases[4], int n_groups, const int32_t* labels,
                                         uint64_t kernel_limit, uint64_t user_limit, uint64_t span_limit) {
  const auto t0 = std::chrono::steady_clock::now();
  AssembleResult res;
  if (n_groups < 0 || (uint32_t)n_groups > L_.group_cap) throw std::invalid_argument("n_groups exceeds group capacity");
  Rec16* ev = reinterpret_cast<Rec16*>(slot + L_.ev_off);
  // 1-2. kernel ring
  defs_.clear();
  if (kernel_) {
    ConsumeStats st = kernel_->consume(ev, L_.sig_cap, defs_, kernel_limit);
    res.n_kernel = (uint32_t)st.events;
    res.n_defs = (uint32_t)st.defs;
    res.discarded = st.discarded;
    res.foreign = st.foreign;
    res.busy_stop = st.busy_stop;
    res.ring_begin = st.begin_pos;
    res.ring_end = st.end_pos;
    tables_->apply_defs(defs_.data(), defs_.size());
  }
  // 3. user-space producers
  uint32_t n = res.n_kernel;
  if (user_) {
    Segment seg[2];
    const int ns = ring_take(user_, user_limit, L_.sig_cap - n, seg);
    uint64_t took = 0;
    for (int s = 0; s < ns; ++s) {
      const EventRec* src = reinterpret_cast<const EventRec*>(user_->records() + seg[s].index * sizeof(EventRec));
      tables_->encode_events(src, seg[s].count, ev + n, bases);
      n += (uint32_t)seg[s].count;
      took += seg[s].count;
    }
    user_->release(took);
    const uint64_t left = user_->size();
    res.user_dropped = (n == L_.sig_cap) ? left : 0;
    res.n_user = (uint32_t)took;
  }
  res.n_events = n;
  // 4. spans
  if (spans_) {
    Segment seg[2];
    const int ns = ring_take(spans_, span_limit, L_.span_cap, seg);
    Span20* sp = reinterpret_cast<Span20*>(slot + L_.sp_off);
    uint64_t took = 0;
    for (int s = 0; s < ns; ++s) {
      const SpanRec64* src = reinterpret_cast<const SpanRec64*>(spans_->records() + seg[s].index * sizeof(SpanRec64));
      tables_->encode_spans(src, seg[s].count, sp + took);
      took += seg[s].count;
    }
    spans_->release(took);
    res.n_spans = (uint32_t)took;
  }
  // 5. context-row patch: as many rows as fit behind the events (the slot reserves row_cap rows;
  // unused event capacity takes more)
  const size_t space = L_.bytes - (L_.ev_off + 16 * (size_t)n);
  size_t fit = space / 20;
  while (fit && row_patch_bytes((uint32_t)fit) > space) --fit;
  fit = std::min<size_t>(fit, tables_->pending_rows());
  if (fit) {
    row_ids_.resize(fit);
    rows_.resize(fit);
    const size_t got = tables_->take_rows(row_ids_.data(), rows_.data(), fit);
    uint8_t* patch = slot + L_.ev_off + 16 * (size_t)n;
    std::memcpy(patch, row_ids_.data(), 4 * got);
    std::memcpy(patch + round16(4 * got), rows_.data(), 16 * got);
    res.n_rows = (uint32_t)got;
  }
  res.rows_deferred = (uint32_t)tables_->pending_rows();
  // head: counts + labels
  int32_t* c = reinterpret_cast<int32_t*>(slot);
  std::memset(c, 0, 4 * kSlotCounts);
  c[0] = (int32_t)n;
  c[1] = (int32_t)res.n_spans;
  c[2] = n_groups;
  c[3] = 0;
  const uint64_t b0 = (uint64_t)bases[0];
  c[4] = (int32_t)(uint32_t)b0;
  c[5] = (int32_t)(uint32_t)(b0 >> 32);
  c[7] = 20;
  for (int k = 1; k < 4; ++k) {
    const uint64_t b = (uint64_t)bases[k];
    c[8 + 2 * (k - 1)] = (int32_t)(uint32_t)b;
    c[9 + 2 * (k - 1)] = (int32_t)(uint32_t)(b >> 32);
  }
  c[14] = (int32_t)res.n_rows;
  int32_t* lab = reinterpret_cast<int32_t*>(slot + 64);
  for (uint32_t g = 0; g < L_.group_cap; ++g) lab[g] = (labels && (int)g < n_groups) ? labels[g] : -1;
  tables_->end_window();
  res.dma_bytes = slot_dma_bytes(L_, n, res.n_rows);
  res.host_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  return res;
}

}  // namespace mislo
