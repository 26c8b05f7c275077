// Native wire encoder (wire.h). Single-threaded per agent stream; ~10 ns per event.
#include "wire.h"

#include <cmath>
#include <cstring>
#include <limits>
#include <stdexcept>

namespace mislo {

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
  std::vector<uint64_t> k;
  std::vector<uint32_t> id, g;
  k.swap(keys_);
  id.swap(ids_);
  g.swap(gens_);
  keys_.assign(cap, 0);
  ids_.assign(cap, 0);
  gens_.assign(cap, 0);
  mask_ = cap - 1;
  size_ = 0;
  for (size_t j = 0; j < k.size(); ++j) {
    if (!k[j] || g[j] < min_gen) continue;
    size_t i = splitmix64(k[j]) & mask_;
    while (keys_[i] != 0) i = (i + 1) & mask_;
    keys_[i] = k[j];
    ids_[i] = id[j];
    gens_[i] = g[j];
    ++size_;
  }
}

uint32_t TraceTable::id(uint64_t tr, uint32_t gen) {
  if (tr == 0) return 0;
  size_t i = splitmix64(tr) & mask_;
  for (;; i = (i + 1) & mask_) {
    if (keys_[i] == tr) {
      gens_[i] = gen;
      return ids_[i];
    }
    if (keys_[i] == 0) break;
  }
  // new trace: ids wrap at 2^32 (skipping 0); a live trace would have to outlast 2^32 newer
  // ones to collide
  const uint32_t v = next_;
  next_ = next_ == 0xFFFFFFFFu ? 1u : next_ + 1;
  keys_[i] = tr;
  ids_[i] = v;
  gens_[i] = gen;
  if (2 * ++size_ > keys_.size()) rehash(keys_.size() * 2, 0);
  return v;
}

void TraceTable::expire(uint32_t min_gen) {
  // rebuild only when the table is large; shrink back if most entries are stale
  if (size_ < (1u << 20)) return;
  size_t live = 0;
  for (size_t j = 0; j < keys_.size(); ++j) live += keys_[j] && gens_[j] >= min_gen;
  size_t cap = 1 << 16;
  while (cap < 4 * live) cap <<= 1;
  rehash(cap, min_gen);
}

// ---- WireEncoder --------------------------------------------------------------------------

WireEncoder::WireEncoder(const double* scale256) {
  for (int t = 0; t < 256; ++t) scale_[t] = scale256[t];
  ctx_rows_.push_back({0u, 0u, 0u, 0u});
  ctx_.insert(0x5bd1e9955bd1e995ull, 0);  // the all-zero context (hash of 0,0,0,0 below)
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

static inline uint64_t ctx_hash(uint32_t pod, uint32_t pid, uint32_t cid, uint32_t sn) {
  if ((pod | pid | cid | sn) == 0) return 0x5bd1e9955bd1e995ull;
  return splitmix64(((uint64_t)pod << 32 | pid) ^ splitmix64((uint64_t)cid << 32 | sn));
}

uint32_t WireEncoder::ctx_id(uint32_t pod, uint32_t pid, uint32_t cid, uint32_t sn) {
  const uint64_t h = ctx_hash(pod, pid, cid, sn);
  uint32_t* v = ctx_.find(h, [&](uint32_t id) {
    const auto& r = ctx_rows_[id];
    return r[0] == pod && r[1] == pid && r[2] == cid && r[3] == sn;
  });
  if (v) return *v;
  const uint32_t id = (uint32_t)ctx_rows_.size();
  if (id >= (1u << 24)) throw std::overflow_error("context id space exhausted");
  ctx_rows_.push_back({pod, pid, cid, sn});
  ctx_.insert(h, id);
  return id;
}

int64_t WireEncoder::encode(const EventRec* ev, size_t n, void* out, int wire) {
  if (wire != 20 && wire != 16) throw std::invalid_argument("wire must be 20 or 16");
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
    const double sc = st < 256 ? scale_[st] : 1.0;
    // records.py _milli_values: rint(value * scale * 1000) clipped to u32 (no FMA:
    // -ffp-contract=off). Adding and subtracting 2^52 rounds half-to-even in the default
    // rounding mode for 0 <= x < 2^52 without a libm call.
    const double x = (double)e.value * sc * 1000.0;
    double milli;
    if (!(x > 0.0)) milli = 0.0;
    else if (x >= 4294967295.0) milli = 4294967295.0;
    else {
      volatile double r = x + 4503599627370496.0;  // volatile: keep the rounding step
      milli = r - 4503599627370496.0;
    }
    const uint32_t cid = conn_id(conn_key(e));
    const uint32_t sn = ((uint32_t)e.svc_id << 16) | e.node_id;
    const uint32_t ctx = ctx_id(e.pod_id, e.pid, cid, sn);
    const uint32_t ct = (st & 0xFFu) | (ctx << 8);
    if (wire == 20) {
      o20[i] = Wire20{ts_off, ct, (uint32_t)milli, (uint32_t)e.trace_h, (uint32_t)(e.trace_h >> 32)};
    } else {
      o16[i] = Wire16{ts_off, ct, (uint32_t)milli, traces_.id(e.trace_h, gen_)};
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

void WireEncoder::end_window() {
  ++gen_;
  if (gen_ > 2) traces_.expire(gen_ - 2);
}

}  // namespace mislo
