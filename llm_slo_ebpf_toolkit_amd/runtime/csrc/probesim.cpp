#include "probesim.h"

#include <cstring>
#include <stdexcept>

namespace mislo {

ProbeSim::ProbeSim(uint64_t* cfg, const int8_t* shift256, size_t trace_lru) : cfg_(cfg), trace_lru_(trace_lru) {
  if (!cfg) throw std::invalid_argument("ProbeSim needs the emulated mislo_cfg array");
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

template <class Emit>
void ProbeSim::one(const EventRec& e, Emit&& emit) {
  const uint32_t st = e.signal_type;
  // mislo_below_floor
  if (st < 120 && e.value < __atomic_load_n(&cfg_[cfg_floor((int)st)], __ATOMIC_RELAXED)) return;
  const uint64_t ck = conn_key(e);
  const uint32_t c32 = conn32(ck);
  uint32_t ctx = 0, tid = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
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
          if (emit(Rec16{c32, kDefCtx | ((uint32_t)fresh << 8), e.pod_id, e.pid})) {
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
        if (emit(Rec16{v, kDefTrace, (uint32_t)e.trace_h, (uint32_t)(e.trace_h >> 32)})) {
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
  emit(r);
}

uint64_t ProbeSim::submit(Ringbuf& rb, const EventRec* ev, size_t n) {
  uint64_t ok = 0;
  for (size_t i = 0; i < n; ++i) {
    bool last_ok = false;
    one(ev[i], [&](const Rec16& r) {
      last_ok = rb.output(&r, sizeof(r));
      if (!last_ok) ++dropped_;
      return last_ok;
    });
    ok += last_ok;
  }
  return ok;
}

void ProbeSim::encode(const EventRec* ev, size_t n, std::vector<Rec16>& out) {
  out.reserve(out.size() + n);
  for (size_t i = 0; i < n; ++i)
    one(ev[i], [&](const Rec16& r) {
      out.push_back(r);
      return true;
    });
}

}  // namespace mislo
