#include "tables.h"

#include <algorithm>
#include <stdexcept>

namespace mislo {

namespace {
inline uint64_t host_hash(uint32_t pod, uint32_t pid, uint32_t c32, uint32_t sn) {
  return splitmix64(((uint64_t)pod << 32 | pid) ^ splitmix64(((uint64_t)c32 << 32) | sn));
}
}  // namespace

AgentTables::AgentTables(const int8_t* shift256) {
  for (int t = 0; t < 256; ++t) {
    if (shift256[t] < -9 || shift256[t] > 9) throw std::invalid_argument("milli shift out of range");
    shift_[t] = shift256[t];
  }
  kernel_rows_.push_back({0u, 0u, 0u, 0u});  // id 0: the all-zero context
  host_.assign(1 << 12, HSlot{0, 0, 0, 0, 0});
  host_mask_ = host_.size() - 1;
  trace_rehash(1 << 16, 0);
}

void AgentTables::queue_row(uint32_t id, const Row& r) { pending_.emplace_back(id, r); }

void AgentTables::set_pod(uint32_t pod, uint32_t svcnode) {
  if (pod >= (1u << 26)) throw std::invalid_argument("pod id out of range");
  if (pod >= pod_sn_.size()) pod_sn_.resize(std::max<size_t>(pod + 1, pod_sn_.size() * 2), 0u);
  if (pod_sn_[pod] == svcnode) return;
  pod_sn_[pod] = svcnode;
  // kernel rows of this pod carry the old svc|node: rewrite them (rare: pod metadata churn)
  for (size_t id = 1; id < kernel_rows_.size(); ++id) {
    Row& r = kernel_rows_[id];
    if (r[0] == pod && (r[0] | r[1] | r[2])) {
      r[3] = svcnode;
      queue_row((uint32_t)id, r);
    }
  }
}

void AgentTables::apply_defs(const Rec16* defs, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const Rec16& d = defs[i];
    const uint32_t type = d.ctx_type & 0xFFu;
    if (type == kDefCtx) {
      const uint32_t id = d.ctx_type >> 8;
      if (id == 0 || id >= kKernelCtxLimit) {
        ++bad_defs_;
        continue;
      }
      if (id >= kernel_rows_.size()) kernel_rows_.resize(id + 1, Row{0u, 0u, 0u, 0u});
      const Row r{d.value_milli, d.trace_tag, d.ts_off, pod_svcnode(d.value_milli)};
      kernel_rows_[id] = r;
      queue_row(id, r);
    } else if (type == kDefTrace) {
      const uint32_t id = d.ts_off;
      if (id == 0 || id >= kKernelTraceLimit) {
        ++bad_defs_;
        continue;
      }
      trace_put((uint64_t)d.value_milli | ((uint64_t)d.trace_tag << 32), id);
    } else {
      ++bad_defs_;
    }
  }
}

// ---- traces ----------------------------------------------------------------------------

void AgentTables::trace_rehash(size_t cap, uint32_t min_gen) {
  std::vector<TSlot> old;
  old.swap(tr_);
  tr_.assign(cap, TSlot{0, 0, 0});
  tr_mask_ = cap - 1;
  tr_size_ = 0;
  for (const TSlot& o : old) {
    if (!o.key || o.gen < min_gen) continue;
    size_t i = splitmix64(o.key) & tr_mask_;
    while (tr_[i].key) i = (i + 1) & tr_mask_;
    tr_[i] = o;
    ++tr_size_;
  }
}

void AgentTables::trace_put(uint64_t hash, uint32_t id) {
  if (!hash) return;
  size_t i = splitmix64(hash) & tr_mask_;
  for (;; i = (i + 1) & tr_mask_) {
    if (tr_[i].key == hash) {  // the kernel's id wins over a host-assigned one
      tr_[i].id = id;
      tr_[i].gen = gen_;
      return;
    }
    if (!tr_[i].key) break;
  }
  tr_[i] = TSlot{hash, id, gen_};
  if (2 * ++tr_size_ > tr_.size()) trace_rehash(tr_.size() * 2, 0);
}

uint32_t AgentTables::trace_id(uint64_t hash) {
  if (!hash) return 0;
  size_t i = splitmix64(hash) & tr_mask_;
  for (;; i = (i + 1) & tr_mask_) {
    if (tr_[i].key == hash) {
      tr_[i].gen = gen_;
      return tr_[i].id;
    }
    if (!tr_[i].key) break;
  }
  const uint32_t v = tr_next_;
  tr_next_ = tr_next_ == kTraceIdMask ? kKernelTraceLimit : tr_next_ + 1;  // host range wraps
  tr_[i] = TSlot{hash, v, gen_};
  if (2 * ++tr_size_ > tr_.size()) trace_rehash(tr_.size() * 2, 0);
  return v;
}

// ---- host contexts ---------------------------------------------------------------------

void AgentTables::host_reset() {
  std::fill(host_.begin(), host_.end(), HSlot{0, 0, 0, 0, 0});
  host_size_ = 0;
  host_next_ = kKernelCtxLimit;
  ++host_wraps_;
}

uint32_t AgentTables::host_ctx(uint32_t pod, uint32_t pid, uint32_t c32, uint32_t sn) {
  if ((pod | pid | c32 | sn) == 0) return 0;
  const uint64_t h = host_hash(pod, pid, c32, sn);
  size_t i = h & host_mask_;
  for (;; i = (i + 1) & host_mask_) {
    const HSlot& s = host_[i];
    if (!s.id) break;
    if (s.pod == pod && s.pid == pid && s.c32 == c32 && s.sn == sn) return s.id;
  }
  if (host_next_ >= kCtxIds) {  // host range exhausted: start over (ids are re-defined as used)
    host_reset();
    i = h & host_mask_;
  }
  if (2 * (host_size_ + 1) > host_.size()) {
    std::vector<HSlot> old;
    old.swap(host_);
    host_.assign(old.size() * 2, HSlot{0, 0, 0, 0, 0});
    host_mask_ = host_.size() - 1;
    for (const HSlot& o : old) {
      if (!o.id) continue;
      size_t j = host_hash(o.pod, o.pid, o.c32, o.sn) & host_mask_;
      while (host_[j].id) j = (j + 1) & host_mask_;
      host_[j] = o;
    }
    i = h & host_mask_;
    while (host_[i].id) i = (i + 1) & host_mask_;
  }
  const uint32_t id = host_next_++;
  host_[i] = HSlot{pod, pid, c32, sn, id};
  ++host_size_;
  queue_row(id, Row{pod, pid, c32, sn});
  return id;
}

size_t AgentTables::encode_events(const EventRec* ev, size_t n, Rec16* out, const int64_t bases[4]) {
  // epoch choice per record: the latest base at or below ts (records a few cuts old keep
  // their own base); a record older than every base clamps to offset 0 of the oldest
  int order[4] = {0, 1, 2, 3};
  std::sort(order, order + 4, [&](int a, int b) { return bases[a] < bases[b]; });
  int oldest = -1;
  for (int k = 0; k < 4; ++k)
    if (bases[order[k]] != 0) {
      oldest = order[k];
      break;
    }
  if (oldest < 0) oldest = 0;
  for (size_t i = 0; i < n; ++i) {
    const EventRec& e = ev[i];
    int tag = oldest;
    for (int k = 3; k >= 0; --k) {
      const int j = order[k];
      if (bases[j] != 0 && e.ts_ns >= bases[j]) {
        tag = j;
        break;
      }
    }
    const uint32_t st = e.signal_type;
    const uint32_t sn = ((uint32_t)e.svc_id << 16) | e.node_id;
    const uint32_t ctx = host_ctx(e.pod_id, e.pid, conn32(conn_key(e)), sn);
    Rec16 r;
    r.ts_off = epoch_offset(e.ts_ns, (uint64_t)bases[tag]);
    r.ctx_type = (st & 0xFFu) | (ctx << 8);
    r.value_milli = milli_int(e.value, st < 256 ? shift_[st] : 3);
    r.trace_tag = (trace_id(e.trace_h) & kTraceIdMask) | ((uint32_t)tag << kEpochTagShift);
    out[i] = r;
  }
  return n;
}

void AgentTables::encode_spans(const SpanRec64* sp, size_t n, Span20* out) {
  for (size_t i = 0; i < n; ++i) {
    const SpanRec64& s = sp[i];
    if (s.group_id < 4096) {
      if (s.group_id >= grp_n_.size()) {
        grp_n_.resize(s.group_id + 1, 0);
        grp_breach_.resize(s.group_id + 1, 0);
      }
      ++grp_n_[s.group_id];
      grp_breach_[s.group_id] += s.ttft_ms > sli_ttft_ms_;
    }
    const uint32_t sn = ((uint32_t)s.svc_id << 16) | s.node_id;
    out[i] = Span20{s.ts_ns, trace_id(s.trace_h), host_ctx(s.pod_id, s.pid, conn32(s.conn_h), sn), s.group_id};
  }
}

size_t AgentTables::take_group_sli(uint32_t* out_n, uint32_t* out_breach, size_t groups) {
  for (size_t g = 0; g < groups; ++g) {
    out_n[g] = g < grp_n_.size() ? grp_n_[g] : 0;
    out_breach[g] = g < grp_breach_.size() ? grp_breach_[g] : 0;
  }
  std::fill(grp_n_.begin(), grp_n_.end(), 0u);
  std::fill(grp_breach_.begin(), grp_breach_.end(), 0u);
  return groups;
}

size_t AgentTables::take_rows(uint32_t* ids, Row* rows, size_t cap) {
  size_t k = 0;
  while (k < cap && pending_head_ < pending_.size()) {
    ids[k] = pending_[pending_head_].first;
    rows[k] = pending_[pending_head_].second;
    ++k;
    ++pending_head_;
  }
  if (pending_head_ == pending_.size()) {
    pending_.clear();
    pending_head_ = 0;
  }
  return k;
}

void AgentTables::end_window() {
  ++gen_;
  // rebuild only when the table is large; entries idle for two windows are dropped
  if (tr_size_ >= (1u << 20) && gen_ > 2) {
    size_t live = 0;
    for (const TSlot& s : tr_) live += s.key && s.gen >= gen_ - 2;
    size_t cap = 1 << 16;
    while (cap < 4 * live) cap <<= 1;
    trace_rehash(cap, gen_ - 2);
  }
}

}  // namespace mislo
