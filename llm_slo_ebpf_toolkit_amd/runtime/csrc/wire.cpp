// Native wire encoder (wire.h): sequential encode()/encode_spans() and the pooled
// encode_window() the agent runs per window.
#include "wire.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <exception>
#include <limits>
#include <stdexcept>

namespace mislo {

static inline uint64_t ctx_hash(uint32_t pod, uint32_t pid, uint64_t ckey, uint32_t sn) {
  if ((pod | pid | sn) == 0 && ckey == 0) return 0x5bd1e9955bd1e995ull;
  return splitmix64(((uint64_t)pod << 32 | pid) ^ splitmix64(ckey ^ ((uint64_t)sn << 7)));
}

// ---- FlatMap ------------------------------------------------------------------------------

FlatMap::FlatMap(size_t cap) {
  size_t c = 16;
  while (c < cap) c <<= 1;
  keys_.assign(c, 0);
  vals_.assign(c, 0);
  mask_ = c - 1;
}

template <class Eq>
uint32_t* FlatMap::find(uint64_t h, Eq eq) {
  h = h ? h : 1;
  for (size_t i = h & mask_;; i = (i + 1) & mask_) {
    if (keys_[i] == 0) return nullptr;
    if (keys_[i] == h && eq(vals_[i])) return &vals_[i];
  }
}

void FlatMap::insert(uint64_t h, uint32_t v) {
  if (2 * (size_ + 1) > keys_.size()) grow();
  h = h ? h : 1;
  size_t i = h & mask_;
  while (keys_[i] != 0) i = (i + 1) & mask_;
  keys_[i] = h;
  vals_[i] = v;
  ++size_;
}

void FlatMap::grow() {
  std::vector<uint64_t> k;
  std::vector<uint32_t> v;
  k.swap(keys_);
  v.swap(vals_);
  keys_.assign(k.size() * 2, 0);
  vals_.assign(k.size() * 2, 0);
  mask_ = keys_.size() - 1;
  for (size_t j = 0; j < k.size(); ++j) {
    if (!k[j]) continue;
    size_t i = k[j] & mask_;
    while (keys_[i] != 0) i = (i + 1) & mask_;
    keys_[i] = k[j];
    vals_[i] = v[j];
  }
}

void FlatMap::clear() {
  std::fill(keys_.begin(), keys_.end(), 0);
  size_ = 0;
}

// ---- TraceTable ---------------------------------------------------------------------------

TraceTable::TraceTable() { rehash(1 << 16, 0); }

void TraceTable::rehash(size_t cap, uint32_t min_gen) {
  std::vector<Slot> old;
  old.swap(slots_);
  slots_.assign(cap, Slot{0, 0, 0});
  mask_ = cap - 1;
  size_ = 0;
  for (const Slot& o : old) {
    if (!o.key || o.gen < min_gen) continue;
    size_t i = splitmix64(o.key) & mask_;
    while (slots_[i].key != 0) i = (i + 1) & mask_;
    slots_[i] = o;
    ++size_;
  }
}

uint32_t TraceTable::id(uint64_t tr, uint32_t gen) {
  if (tr == 0) return 0;
  size_t i = splitmix64(tr) & mask_;
  for (;; i = (i + 1) & mask_) {
    if (slots_[i].key == tr) {
      slots_[i].gen = gen;
      return slots_[i].id;
    }
    if (slots_[i].key == 0) break;
  }
  // new trace: ids wrap at 2^30 (skipping 0; EVENT16 keeps the top 2 bits for the epoch tag);
  // a live trace would have to outlast 2^30 newer ones to collide
  const uint32_t v = next_;
  next_ = next_ == kTraceIdMask ? 1u : next_ + 1;
  slots_[i] = Slot{tr, v, gen};
  if (2 * ++size_ > slots_.size()) rehash(slots_.size() * 2, 0);
  return v;
}

uint32_t TraceTable::find_touch(uint64_t tr, uint32_t gen) {
  if (tr == 0) return 0;
  for (size_t i = splitmix64(tr) & mask_;; i = (i + 1) & mask_) {
    Slot& sl = slots_[i];
    if (sl.key == tr) {
      if (__atomic_load_n(&sl.gen, __ATOMIC_RELAXED) != gen) __atomic_store_n(&sl.gen, gen, __ATOMIC_RELAXED);
      return sl.id;
    }
    if (sl.key == 0) return 0;
  }
}

void TraceTable::expire(uint32_t min_gen) {
  // rebuild only when the table is large; shrink back if most entries are stale
  if (size_ < (1u << 20)) return;
  size_t live = 0;
  for (const Slot& sl : slots_) live += sl.key && sl.gen >= min_gen;
  size_t cap = 1 << 16;
  while (cap < 4 * live) cap <<= 1;
  rehash(cap, min_gen);
}

// ---- CtxMap -------------------------------------------------------------------------------

CtxMap::CtxMap(size_t cap) {
  size_t c = 16;
  while (c < cap) c <<= 1;
  slots_.assign(c, Slot{0, 0, 0, 0, kEmpty});
  mask_ = c - 1;
}

uint32_t CtxMap::find(uint64_t h, uint64_t ppid, uint64_t ck, uint32_t sn) const {
  for (size_t i = h & mask_;; i = (i + 1) & mask_) {
    const Slot& sl = slots_[i];
    if (sl.id == kEmpty) return kEmpty;
    if (sl.ppid == ppid && sl.ck == ck && sl.sn == sn) return sl.id;
  }
}

void CtxMap::insert(uint64_t h, uint64_t ppid, uint64_t ck, uint32_t sn, uint32_t id) {
  if (2 * (size_ + 1) > slots_.size()) {
    std::vector<Slot> old;
    old.swap(slots_);
    slots_.assign(old.size() * 2, Slot{0, 0, 0, 0, kEmpty});
    mask_ = slots_.size() - 1;
    for (const Slot& o : old) {
      if (o.id == kEmpty) continue;
      size_t i = o.h & mask_;
      while (slots_[i].id != kEmpty) i = (i + 1) & mask_;
      slots_[i] = o;
    }
  }
  size_t i = h & mask_;
  while (slots_[i].id != kEmpty) i = (i + 1) & mask_;
  slots_[i] = Slot{ppid, ck, h, sn, id};
  ++size_;
}

void CtxMap::clear() {
  for (Slot& sl : slots_) sl.id = kEmpty;
  size_ = 0;
}

// ---- WireEncoder --------------------------------------------------------------------------

WireEncoder::WireEncoder(const int8_t* shift256) {
  for (int t = 0; t < 256; ++t) {
    if (shift256[t] < -9 || shift256[t] > 9) throw std::invalid_argument("milli shift out of range");
    shift_[t] = shift256[t];
  }
  ctx_rows_.push_back({0u, 0u, 0u, 0u});
  ctx_.insert(ctx_hash(0, 0, 0, 0), 0, 0, 0, 0);  // the all-zero context
}

uint32_t WireEncoder::conn_id(uint64_t key) {
  if (key == 0) return 0;
  uint32_t* v = conns_.find(key, [](uint32_t) { return true; });
  if (v) return *v;
  const uint32_t id = (uint32_t)(++n_conns_);
  if (id >= (1u << 24)) throw std::overflow_error("connection id space exhausted");
  conns_.insert(key, id);
  return id;
}

uint32_t WireEncoder::conn_find(uint64_t key) {
  uint32_t* v = conns_.find(key, [](uint32_t) { return true; });
  return v ? *v : 0;
}

uint32_t WireEncoder::ctx_find(uint32_t pod, uint32_t pid, uint64_t ckey, uint32_t sn) {
  return ctx_.find(ctx_hash(pod, pid, ckey, sn), (uint64_t)pod << 32 | pid, ckey, sn);
}

uint32_t WireEncoder::ctx_id(uint32_t pod, uint32_t pid, uint64_t ckey, uint32_t sn) {
  const uint64_t h = ctx_hash(pod, pid, ckey, sn), ppid = (uint64_t)pod << 32 | pid;
  const uint32_t found = ctx_.find(h, ppid, ckey, sn);
  if (found != kAbsent) return found;
  const uint32_t id = (uint32_t)ctx_rows_.size();
  if (id >= (1u << 24)) throw std::overflow_error("context id space exhausted");
  const uint32_t cid = ckey ? conn_id(ckey) : 0;
  ctx_rows_.push_back({pod, pid, cid, sn});
  ctx_.insert(h, ppid, ckey, sn, id);
  return id;
}

int64_t WireEncoder::encode(const EventRec* ev, size_t n, void* out, int wire) {
  if (wire == 32) {
    Event32* o = static_cast<Event32*>(out);
    for (size_t i = 0; i < n; ++i) {
      const EventRec& e = ev[i];
      const uint32_t st = e.signal_type;
      const uint64_t ck = conn_key(e);
      const uint32_t cid = ck ? conn_id(ck) : 0;
      o[i] = Event32{e.ts_ns, e.trace_h, milli_int(e.value, st < 256 ? shift_[st] : 3), e.pid, e.pod_id,
                     (st & 0xFFu) | (cid << 8)};
    }
    return 0;
  }
  if (wire == 24) {
    Event24* o = static_cast<Event24*>(out);
    for (size_t i = 0; i < n; ++i) {
      const EventRec& e = ev[i];
      const uint32_t st = e.signal_type;
      const uint64_t ck = conn_key(e);
      if (ck) conn_id(ck);
      const uint32_t ctx = ctx_id(e.pod_id, e.pid, ck, ((uint32_t)e.svc_id << 16) | e.node_id);
      o[i] = Event24{e.ts_ns, e.trace_h, milli_int(e.value, st < 256 ? shift_[st] : 3), (st & 0xFFu) | (ctx << 8)};
    }
    return 0;
  }
  if (wire == kWire20T) {
    Event20T* o = static_cast<Event20T*>(out);
    for (size_t i = 0; i < n; ++i) {
      const EventRec& e = ev[i];
      const uint32_t st = e.signal_type;
      const uint64_t ck = conn_key(e);
      if (ck) conn_id(ck);
      const uint32_t ctx = ctx_id(e.pod_id, e.pid, ck, ((uint32_t)e.svc_id << 16) | e.node_id);
      o[i] = Event20T{e.ts_ns, milli_int(e.value, st < 256 ? shift_[st] : 3), (st & 0xFFu) | (ctx << 8),
                      traces_.id(e.trace_h, gen_)};
    }
    return 0;
  }
  if (wire != 20 && wire != 16) throw std::invalid_argument("wire must be 32, 24, 21, 20 or 16");
  int64_t t_base = std::numeric_limits<int64_t>::max(), t_max = std::numeric_limits<int64_t>::min();
  for (size_t i = 0; i < n; ++i) {
    const int64_t t = ev[i].ts_ns;
    if (t == 0) continue;
    t_base = t < t_base ? t : t_base;
    t_max = t > t_max ? t : t_max;
  }
  if (t_max == std::numeric_limits<int64_t>::min()) t_base = 0;
  else if ((uint64_t)(t_max - t_base) >= (uint64_t)kWireTsZero)
    throw std::range_error("window spans >= 2^32 ns: not representable in the 20/16-byte wire format");
  Wire20* o20 = static_cast<Wire20*>(out);
  Wire16* o16 = static_cast<Wire16*>(out);
  for (size_t i = 0; i < n; ++i) {
    const EventRec& e = ev[i];
    const uint32_t ts_off = e.ts_ns == 0 ? kWireTsZero : (uint32_t)(e.ts_ns - t_base);
    const uint32_t st = e.signal_type;
    const uint32_t milli = milli_int(e.value, st < 256 ? shift_[st] : 3);
    const uint64_t ck = conn_key(e);
    if (ck) conn_id(ck);  // ids in event order (the context row refers to it)
    const uint32_t sn = ((uint32_t)e.svc_id << 16) | e.node_id;
    const uint32_t ctx = ctx_id(e.pod_id, e.pid, ck, sn);
    const uint32_t ct = (st & 0xFFu) | (ctx << 8);
    if (wire == 20) {
      o20[i] = Wire20{ts_off, ct, milli, (uint32_t)e.trace_h, (uint32_t)(e.trace_h >> 32)};
    } else {
      o16[i] = Wire16{ts_off, ct, milli, traces_.id(e.trace_h, gen_)};
    }
  }
  return t_base;
}

void WireEncoder::encode_spans(const SpanRec64* in, size_t n, SpanRec64* out, bool trace_ids) {
  for (size_t i = 0; i < n; ++i) {
    SpanRec64 s = in[i];
    s.conn_h = conn_id(s.conn_h);
    if (trace_ids) s.trace_h = traces_.id(s.trace_h, gen_);
    out[i] = s;
  }
}

void WireEncoder::encode_spans20(const SpanRec64* in, size_t n, Span20* out) {
  for (size_t i = 0; i < n; ++i) {
    const SpanRec64& s = in[i];
    const uint32_t ctx = ctx_id(s.pod_id, s.pid, s.conn_h, ((uint32_t)s.svc_id << 16) | s.node_id);
    out[i] = Span20{s.ts_ns, traces_.id(s.trace_h, gen_), ctx, s.group_id};
  }
}

void WireEncoder::end_window() {
  ++gen_;
  if (gen_ > 2) traces_.expire(gen_ - 2);
}

// ---- WorkerPool ---------------------------------------------------------------------------

WorkerPool::WorkerPool(int threads) {
  for (int i = 1; i < std::max(1, threads); ++i) workers_.emplace_back([this] { loop(); });
}

WorkerPool::~WorkerPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void WorkerPool::drain_tasks() {
  for (;;) {
    const int i = next_.fetch_add(1, std::memory_order_relaxed);
    if (i >= ntasks_) return;
    (*fn_)(i);
    std::lock_guard<std::mutex> g(mu_);
    if (--pending_ == 0) done_cv_.notify_all();
  }
}

void WorkerPool::loop() {
  uint64_t seen = 0;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || epoch_ != seen; });
      if (stop_) return;
      seen = epoch_;
    }
    drain_tasks();
  }
}

void WorkerPool::run(int ntasks, const std::function<void(int)>& fn) {
  if (ntasks <= 0) return;
  if (workers_.empty() || ntasks == 1) {
    for (int i = 0; i < ntasks; ++i) fn(i);
    return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    fn_ = &fn;
    ntasks_ = ntasks;
    pending_ = ntasks;
    next_.store(0, std::memory_order_relaxed);
    ++epoch_;
  }
  cv_.notify_all();
  drain_tasks();
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return pending_ == 0; });
  // a worker woken late finds next_ >= ntasks_ and goes back to sleep; fn_ stays valid
  // until the next run() replaces it under the lock
}

// ---- encode_window ------------------------------------------------------------------------

void ChunkScratch::reset() {
  tmin = std::numeric_limits<int64_t>::max();
  tmax = std::numeric_limits<int64_t>::min();
  if (conn_map.size()) conn_map.clear();
  if (ctx_map.size()) ctx_map.clear();
  if (trace_map.size()) trace_map.clear();
  new_conns.clear();
  new_traces.clear();
  new_ctx.clear();
  fix.clear();
}

static inline uint32_t local_index(FlatMap& m, std::vector<uint64_t>& list, uint64_t key) {
  uint32_t* v = m.find(key, [&](uint32_t j) { return list[j] == key; });
  if (v) return *v;
  const uint32_t j = (uint32_t)list.size();
  list.push_back(key);
  m.insert(key, j);
  return j;
}

void WireEncoder::encode_chunk(const EventRec* ev, size_t lo, size_t hi, int64_t base, void* out, int wire,
                               ChunkScratch& cs) {
  Wire20* o20 = static_cast<Wire20*>(out);
  Wire16* o16 = static_cast<Wire16*>(out);
  int64_t tmin = cs.tmin, tmax = cs.tmax;
  // consecutive events often repeat a context / trace: remember the last resolution
  bool have_last = false;
  uint64_t last_ppid = 0, last_ck = 0;
  uint32_t last_sn = 0, last_ctx = 0, last_ctx_fix = 0;
  uint64_t last_tr = 0;
  uint32_t last_tid = 0, last_tr_fix = 0;
  for (size_t i = lo; i < hi; ++i) {
    const EventRec& e = ev[i];
    const int64_t t = e.ts_ns;
    uint32_t ts_off = kWireTsZero;
    if (t != 0) {
      tmin = t < tmin ? t : tmin;
      tmax = t > tmax ? t : tmax;
      ts_off = (uint32_t)(uint64_t)(t - base);  // rebased in phase 3 if base is not the minimum
    }
    const uint32_t st = e.signal_type;
    const uint32_t milli = milli_int(e.value, st < 256 ? shift_[st] : 3);
    const uint64_t ck = conn_key(e);
    const uint64_t ppid = (uint64_t)e.pod_id << 32 | e.pid;
    const uint32_t sn = ((uint32_t)e.svc_id << 16) | e.node_id;
    uint32_t fixbits = 0;
    if (!(have_last && ppid == last_ppid && ck == last_ck && sn == last_sn)) {
      have_last = true;
      const uint64_t h = ctx_hash(e.pod_id, e.pid, ck, sn);
      uint32_t c = ctx_.find(h, ppid, ck, sn);
      last_ctx_fix = 0;
      if (c == kAbsent) {
        // a known context implies a known connection; only new contexts can bring new ones
        if (ck && conn_find(ck) == 0) local_index(cs.conn_map, cs.new_conns, ck);
        c = cs.ctx_map.find(h, ppid, ck, sn);
        if (c == kAbsent) {
          c = (uint32_t)cs.new_ctx.size();
          if (c >= (1u << 24)) throw std::overflow_error("context id space exhausted");
          cs.new_ctx.push_back({ppid, ck, sn});
          cs.ctx_map.insert(h, ppid, ck, sn, c);
        }
        last_ctx_fix = 1;
      }
      last_ppid = ppid, last_ck = ck, last_sn = sn, last_ctx = c;
    }
    fixbits |= last_ctx_fix;
    const uint32_t ct = (st & 0xFFu) | (last_ctx << 8);
    if (wire == 20) {
      o20[i] = Wire20{ts_off, ct, milli, (uint32_t)e.trace_h, (uint32_t)(e.trace_h >> 32)};
    } else {
      const uint64_t tr = e.trace_h;
      if (tr != last_tr || i == lo) {
        last_tid = traces_.find_touch(tr, gen_);
        last_tr_fix = 0;
        if (tr != 0 && last_tid == 0) {
          last_tid = local_index(cs.trace_map, cs.new_traces, tr);
          last_tr_fix = 2;
        }
        last_tr = tr;
      }
      fixbits |= last_tr_fix;
      o16[i] = Wire16{ts_off, ct, milli, last_tid};
    }
    if (fixbits) cs.fix.push_back((uint64_t)i << 2 | fixbits);
  }
  cs.tmin = tmin;
  cs.tmax = tmax;
}

void WireEncoder::spans_chunk(const SpanRec64* sp, size_t lo, size_t hi, SpanRec64* out, bool trace_ids,
                              ChunkScratch& cs) {
  for (size_t i = lo; i < hi; ++i) {
    SpanRec64 s = sp[i];
    uint32_t fixbits = 0;
    if (s.conn_h) {
      const uint32_t c = conn_find(s.conn_h);
      if (c) {
        s.conn_h = c;
      } else {
        s.conn_h = local_index(cs.conn_map, cs.new_conns, s.conn_h);
        fixbits |= 1;
      }
    }
    if (trace_ids && s.trace_h) {
      const uint32_t t = traces_.find_touch(s.trace_h, gen_);
      if (t) {
        s.trace_h = t;
      } else {
        s.trace_h = local_index(cs.trace_map, cs.new_traces, s.trace_h);
        fixbits |= 2;
      }
    }
    out[i] = s;
    if (fixbits) cs.fix.push_back((uint64_t)i << 2 | fixbits);
  }
}

int64_t WireEncoder::encode_window(const EventRec* ev, size_t n, void* ev_out, int wire, const SpanRec64* sp,
                                   size_t n_sp, SpanRec64* sp_out, int threads, size_t min_chunk) {
  if (wire != 20 && wire != 16) throw std::invalid_argument("wire must be 20 or 16");
  threads = std::max(1, std::min(threads, 64));
  if (!pool_ || pool_->threads() != threads) pool_ = std::make_unique<WorkerPool>(threads);
  // chunking: contiguous ranges of >= min_chunk events / min_chunk / 8 spans; event chunks
  // first, then spans
  const size_t kEv = std::max<size_t>(1, min_chunk), kSp = std::max<size_t>(1, min_chunk / 8);
  const int ce = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads * 2, (n + kEv - 1) / kEv));
  const int csn = n_sp ? (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, (n_sp + kSp - 1) / kSp)) : 0;
  const int nc = ce + csn;
  if ((int)chunks_.size() < nc) chunks_.resize(nc);
  auto ev_range = [&](int c) { return std::make_pair(n * c / ce, n * (c + 1) / ce); };
  auto sp_range = [&](int c) { return std::make_pair(n_sp * c / csn, n_sp * (c + 1) / csn); };
  int64_t base = 0;  // provisional t_base: the first non-zero timestamp (the minimum if sorted)
  for (size_t i = 0; i < n; ++i)
    if (ev[i].ts_ns) {
      base = ev[i].ts_ns;
      break;
    }
  const bool tr16 = wire == 16;
  // phase 1: chunks (global tables are read-only here). A chunk's exception is rethrown on
  // the calling thread.
  std::vector<std::exception_ptr> errs(nc);
  pool_->run(nc, [&](int c) {
    try {
      ChunkScratch& cs = chunks_[c];
      cs.reset();
      if (c < ce) {
        auto r = ev_range(c);
        encode_chunk(ev, r.first, r.second, base, ev_out, wire, cs);
      } else {
        auto r = sp_range(c - ce);
        spans_chunk(sp, r.first, r.second, sp_out, tr16, cs);
      }
    } catch (...) {
      errs[c] = std::current_exception();
    }
  });
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
  int64_t t_base = std::numeric_limits<int64_t>::max(), t_max = std::numeric_limits<int64_t>::min();
  for (int c = 0; c < ce; ++c) {
    t_base = std::min(t_base, chunks_[c].tmin);
    t_max = std::max(t_max, chunks_[c].tmax);
  }
  if (t_max == std::numeric_limits<int64_t>::min()) t_base = base = 0;
  else if ((uint64_t)(t_max - t_base) >= (uint64_t)kWireTsZero)
    throw std::range_error("window spans >= 2^32 ns: not representable in the 20/16-byte wire format");
  // phase 2 (serial): new keys in chunk order = global first-occurrence order. Events come
  // before spans, exactly as encode() then encode_spans() assign ids.
  for (int c = 0; c < nc; ++c) {
    ChunkScratch& cs = chunks_[c];
    cs.conn_remap.resize(cs.new_conns.size());
    for (size_t j = 0; j < cs.new_conns.size(); ++j) cs.conn_remap[j] = conn_id(cs.new_conns[j]);
    if (c < ce) {
      cs.ctx_remap.resize(cs.new_ctx.size());
      for (size_t j = 0; j < cs.new_ctx.size(); ++j) {
        const auto& k = cs.new_ctx[j];
        cs.ctx_remap[j] = ctx_id((uint32_t)(k[0] >> 32), (uint32_t)k[0], k[1], (uint32_t)k[2]);
      }
    }
    cs.trace_remap.resize(cs.new_traces.size());
    for (size_t j = 0; j < cs.new_traces.size(); ++j) cs.trace_remap[j] = traces_.id(cs.new_traces[j], gen_);
  }
  // phase 3: global ids into the fix-up records; rebase timestamps if needed
  const bool rebase = t_base != base;
  pool_->run(nc, [&](int c) {
    ChunkScratch& cs = chunks_[c];
    if (c < ce) {
      Wire20* o20 = static_cast<Wire20*>(ev_out);
      Wire16* o16 = static_cast<Wire16*>(ev_out);
      for (uint64_t f : cs.fix) {
        const size_t i = f >> 2;
        uint32_t& ct = tr16 ? o16[i].ctx_type : o20[i].ctx_type;
        if (f & 1) ct = (ct & 0xFFu) | (cs.ctx_remap[ct >> 8] << 8);
        if (f & 2) o16[i].trace_id = cs.trace_remap[o16[i].trace_id];
      }
      if (rebase) {
        auto r = ev_range(c);
        for (size_t i = r.first; i < r.second; ++i) {
          const int64_t t = ev[i].ts_ns;
          const uint32_t off = t == 0 ? kWireTsZero : (uint32_t)(t - t_base);
          if (tr16) o16[i].ts_off = off;
          else o20[i].ts_off = off;
        }
      }
    } else {
      for (uint64_t f : cs.fix) {
        SpanRec64& s = sp_out[f >> 2];
        if (f & 1) s.conn_h = cs.conn_remap[s.conn_h];
        if (f & 2) s.trace_h = cs.trace_remap[s.trace_h];
      }
    }
  });
  return t_base;
}

}  // namespace mislo
