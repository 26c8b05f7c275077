#include "probesim.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace mislo {

ProbeSim::ProbeSim(uint64_t* cfg, const int8_t* shift256, size_t trace_lru, uint32_t cpus)
    : cfg_(cfg), trace_lru_(trace_lru), stages_(std::max<uint32_t>(1, cpus)) {
  if (!cfg) throw std::invalid_argument("ProbeSim needs the emulated mislo_cfg array");
  for (Stage& st : stages_)
    for (Rec16& r : st.slot) r = pad_slot();
  for (int t = 0; t < 256; ++t) {
    if (shift256[t] < -9 || shift256[t] > 9) throw std::invalid_argument("milli shift out of range");
    shift_[t] = shift256[t];
  }
}

void ProbeSim::reset_maps() {
  std::lock_guard<std::mutex> g(mu_);
  traces_.clear();
  ctx_.clear();
  __atomic_store_n(&cfg_[kCfgCtxNext], 0, __ATOMIC_RELAXED);
}

// `out(batch)` puts 8 slots on the ring (true = written)
template <class Out>
bool ProbeSim::flush_stage(Stage& st, Out&& out) {
  const uint32_t n_ev = [&] {
    uint32_t c = 0;
    for (uint32_t j = 0; j < st.n; ++j) c += (st.slot[j].ctx_type & 0xFFu) < kDefFirst;
    return c;
  }();
  const bool ok = out(st.slot, n_ev);
  if (!ok) dropped_ += n_ev;
  ++batches_;
  for (Rec16& r : st.slot) r = pad_slot();
  st.n = 0;
  return ok;
}

template <class Out>
bool ProbeSim::put(uint32_t cpu, const Rec16& r, bool def, Out&& out) {
  Stage& st = stages_[cpu % stages_.size()];
  const uint64_t epoch = __atomic_load_n(&cfg_[kCfgEpoch], __ATOMIC_ACQUIRE);
  if (st.n && st.epoch != epoch) flush_stage(st, out);  // a batch holds one epoch's slots
  st.slot[st.n++] = r;
  st.epoch = epoch;
  if (st.n == kBatchSlots || def) return flush_stage(st, out);
  return true;
}

template <class Out>
void ProbeSim::one(const EventRec& e, Out&& out) {
  const uint32_t cpu = e.tid;
  auto emit = [&](const Rec16& r, bool def) { return put(cpu, r, def, out); };
  const uint32_t st = e.signal_type;
  // mislo_below_floor
  if (st < 120 && e.value < __atomic_load_n(&cfg_[cfg_floor((int)st)], __ATOMIC_RELAXED)) return;
  const uint64_t ck = conn_key(e);
  const uint32_t c32 = conn32(ck);
  uint32_t ctx = 0, tid = 0;
  {  // (callers hold mu_: maps and batches)
    if (e.pod_id | e.pid | c32) {
      const CtxKey k{e.pod_id, e.pid, c32};
      auto it = ctx_.find(k);
      if (it != ctx_.end()) {
        ctx = it->second;
      } else {
        const uint64_t fresh = __atomic_fetch_add(&cfg_[kCfgCtxNext], 1, __ATOMIC_RELAXED) + 1;
        if (fresh < kKernelCtxLimit) {
          // definition first, then the map insert (mislo_probe.h MISLO_INTERN_DEF)
          // (a definition the ring dropped leaves the context unnamed: id 0 for this event)
          if (emit(Rec16{c32, kDefCtx | ((uint32_t)fresh << 8), e.pod_id, e.pid}, true)) {
            ctx_.emplace(k, (uint32_t)fresh);
            ctx = (uint32_t)fresh;
          }
        }
      }
    }
    if (e.trace_h) {
      auto it = traces_.find(e.trace_h);
      if (it != traces_.end()) {
        tid = it->second;
      } else {
        const uint64_t fresh = __atomic_fetch_add(&cfg_[kCfgTraceNext], 1, __ATOMIC_RELAXED);
        const uint32_t v = (uint32_t)(fresh % (kKernelTraceLimit - 1)) + 1;
        if (emit(Rec16{v, kDefTrace, (uint32_t)e.trace_h, (uint32_t)(e.trace_h >> 32)}, true)) {
          if (traces_.size() >= trace_lru_) traces_.clear();  // coarse LRU eviction
          traces_.emplace(e.trace_h, v);
          tid = v;
        }
      }
    }
  }
  const uint64_t epoch = __atomic_load_n(&cfg_[kCfgEpoch], __ATOMIC_ACQUIRE);
  Rec16 r;
  r.ts_off = epoch_offset(e.ts_ns, epoch & ~3ull);
  r.ctx_type = (st & 0xFFu) | (ctx << 8);
  r.value_milli = milli_int(e.value, st < 256 ? shift_[st] : 3);
  r.trace_tag = (tid & kTraceIdMask) | ((uint32_t)(epoch & 3) << kEpochTagShift);
  emit(r, false);
}

uint64_t ProbeSim::submit(Ringbuf& rb, const EventRec* ev, size_t n, bool flush_after) {
  uint64_t ok = 0;
  auto out = [&](const Rec16* b, uint32_t n_ev) {
    const bool w = rb.output(b, kRecPayload);
    if (w) ok += n_ev;
    return w;
  };
  {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < n; ++i) one(ev[i], out);
  }
  if (flush_after) ok += flush(rb);
  return ok;
}

uint64_t ProbeSim::flush(Ringbuf& rb) {
  std::lock_guard<std::mutex> g(mu_);
  uint64_t ok = 0;
  for (Stage& st : stages_)
    if (st.n)
      flush_stage(st, [&](const Rec16* b, uint32_t n_ev) {
        const bool w = rb.output(b, kRecPayload);
        if (w) ok += n_ev;
        return w;
      });
  return ok;
}

void ProbeSim::encode(const EventRec* ev, size_t n, std::vector<Rec16>& out, bool flush_after) {
  out.reserve(out.size() + n + n / 4);
  auto put_out = [&](const Rec16* b, uint32_t) {
    out.insert(out.end(), b, b + kBatchSlots);
    return true;
  };
  {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < n; ++i) one(ev[i], put_out);
  }
  if (flush_after) encode_flush(out);
}

void ProbeSim::encode_flush(std::vector<Rec16>& out) {
  std::lock_guard<std::mutex> g(mu_);
  for (Stage& st : stages_)
    if (st.n)
      flush_stage(st, [&](const Rec16* b, uint32_t) {
        out.insert(out.end(), b, b + kBatchSlots);
        return true;
      });
}

}  // namespace mislo
