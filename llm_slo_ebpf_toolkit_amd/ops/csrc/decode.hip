// K1: batched record decode + status + per-signal histograms + join-partition counts.
//
// One pass over the window's 64-byte records (one cache line per event, read as
// 4 x dwordx4 per lane, fully coalesced). Produces the structure-of-arrays columns the
// join and posterior kernels consume, and -- fused into the same pass -- the per-signal
// Prometheus-style histograms (REF agent histogram cmd/agent/main.go:190-194 generalised
// to all 16 signals), per-signal status counters (REF generator.go:203-232 thresholds)
// and the 4 x 1024 hash-partition histograms that size the join's partition buffers.
// All histograms are LDS-privatised per workgroup: signal/status bins are merged with
// one global atomic per non-zero bin (O(bins x workgroups), not O(N)); the partition
// histogram is stored per workgroup for the atomic-free scatter (join.hip).
//
// The REF-compat variant decodes REF's packed 40-byte record with REF's exact unit
// rules (pkg/collector/ringbuf.go:199-238) for replaying REF ring-buffer captures.
#include "mislo_common.h"
#include "mislo_launch.h"
#include <stdexcept>

namespace mislo {

__constant__ Tables c_tab;

struct DecodeOut {
  SignalCols cols;
  uint32_t* hist;        // [kSlots * kBuckets]
  uint32_t* status_cnt;  // [kSlots * 3]
  uint32_t* part_cnt;    // [gridDim.x][kKeyTypes * kParts] per-block partition counts
  unsigned long long* misc;  // [0] unsupported events, [1] zero-timestamp events,
                             // [2 + slot] per-signal value sum in 1/1000 units (Prometheus _sum)
  int blk_base = 0;      // this launch's first row in part_cnt (a second row segment's decode)
  // the exchange's trace-row selection, fused (segment 0 with the exchange): per block the
  // count of selected local rows, per (block, trip, wave) the 64-row ballot mask (exchange.hip
  // k_sel_scatter_mask reads them in the same geometry)
  uint32_t* sel_cnt = nullptr;
  unsigned long long* sel_mask = nullptr;
  int sel_stride = 0;    // masks per block
};

constexpr int kMiscSums = 2;  // offset of the per-slot value sums in misc

// Per-block partition histogram, stored (not atomically merged): the scan kernel turns
// the [blocks][4][1024] matrix into per-block scatter offsets, so the scatter pass needs
// no global atomics and places each block's events contiguously.
template <int NT>
__device__ __forceinline__ void store_counts(const uint32_t* lds, uint32_t* dst) {
  for (int i = threadIdx.x; i < kKeyTypes * kParts; i += NT) dst[i] = lds[i];
}

// LDS counters of one decode workgroup. The small hot arrays (16 x 16 histogram bins, 16 x 3
// status bins, 16 value sums) take an atomic from EVERY event, and a wave's 64 events land on
// a handful of bins: same-address LDS atomics serialise (PMC: 64 % extra LDS cycles with one
// copy). Each lane adds into copy (lane & 7) and the copies are summed at the flush; the odd
// copy strides put the copies of a bin on different banks. The partition histogram (4 x kParts
// hashed bins) gets kPartRep copies too: the pod / service keys of a wave's events repeat (a
// few hundred pods, tens of services), and with kParts = 128 trace keys collide as well.
struct DecodeLds {
  // the signal tables, copied from constant memory once per workgroup: per-event lookups use
  // a lane-varying slot, which constant memory serves as one vector load per element (15 bucket
  // edges + thresholds + type map per event); from LDS a slot's edges are 4 ds_read_b128
  alignas(16) Tables tab;
  static constexpr int kRep = 8, kPartRep = 4;
  static constexpr int kHS = kSlots * kBuckets + 1, kSS = kSlots * 3 + 1, kUS = kSlots + 1;
  static constexpr int kPS = kKeyTypes * kParts + 1;
  uint32_t hist[kRep * kHS];
  uint32_t status[kRep * kSS];
  uint32_t part[kPartRep * kPS];
  unsigned long long sum[kRep * kUS];
};

template <int NT>
__device__ __forceinline__ void lds_init(DecodeLds& L) {
  static_assert(sizeof(Tables) % 4 == 0 && offsetof(Tables, edges) % 16 == 0, "table layout");
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&c_tab);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&L.tab);
    for (int i = threadIdx.x; i < (int)(sizeof(Tables) / 4); i += NT) dst[i] = src[i];
  }
  for (int i = threadIdx.x; i < DecodeLds::kPartRep * DecodeLds::kPS; i += NT) L.part[i] = 0;
  for (int i = threadIdx.x; i < DecodeLds::kRep * DecodeLds::kUS; i += NT) L.sum[i] = 0;
  for (int i = threadIdx.x; i < DecodeLds::kRep * DecodeLds::kHS; i += NT) L.hist[i] = 0;
  for (int i = threadIdx.x; i < DecodeLds::kRep * DecodeLds::kSS; i += NT) L.status[i] = 0;
  __syncthreads();
}

// this lane's copies
struct LdsLane {
  uint32_t *hist, *status, *part;
  unsigned long long* sum;
  const Tables* tab;
};
__device__ __forceinline__ LdsLane lds_lane(DecodeLds& L) {
  const int r = threadIdx.x & (DecodeLds::kRep - 1), q = threadIdx.x & (DecodeLds::kPartRep - 1);
  return LdsLane{L.hist + r * DecodeLds::kHS, L.status + r * DecodeLds::kSS, L.part + q * DecodeLds::kPS,
                 L.sum + r * DecodeLds::kUS, &L.tab};
}

// sum the copies: signal / status bins and value sums merge with one global atomic per
// non-zero bin; the partition counts are stored per workgroup (atomic-free scatter)
template <int NT>
__device__ __forceinline__ void lds_flush(DecodeLds& L, const DecodeOut& o, int unsupported, int zero_ts) {
  __syncthreads();
  for (int i = threadIdx.x; i < kSlots * kBuckets; i += NT) {
    uint32_t v = 0;
#pragma unroll
    for (int r = 0; r < DecodeLds::kRep; ++r) v += L.hist[r * DecodeLds::kHS + i];
    if (v) atomicAdd(o.hist + i, v);
  }
  for (int i = threadIdx.x; i < kSlots * 3; i += NT) {
    uint32_t v = 0;
#pragma unroll
    for (int r = 0; r < DecodeLds::kRep; ++r) v += L.status[r * DecodeLds::kSS + i];
    if (v) atomicAdd(o.status_cnt + i, v);
  }
  if (threadIdx.x < kSlots) {
    unsigned long long v = 0;
#pragma unroll
    for (int r = 0; r < DecodeLds::kRep; ++r) v += L.sum[r * DecodeLds::kUS + threadIdx.x];
    if (v) atomicAdd(&o.misc[kMiscSums + threadIdx.x], v);
  }
  uint32_t* dst = o.part_cnt + (size_t)(o.blk_base + blockIdx.x) * kKeyTypes * kParts;
  for (int i = threadIdx.x; i < kKeyTypes * kParts; i += NT) {
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < DecodeLds::kPartRep; ++q) v += L.part[q * DecodeLds::kPS + i];
    dst[i] = v;
  }
  // wave-level reduction of the scalar counters, one atomic per wave
  for (int off = 32; off > 0; off >>= 1) {
    unsupported += __shfl_xor(unsupported, off);
    zero_ts += __shfl_xor(zero_ts, off);
  }
  if ((threadIdx.x & 63) == 0) {
    if (unsupported) atomicAdd(&o.misc[0], (unsigned long long)unsupported);
    if (zero_ts) atomicAdd(&o.misc[1], (unsigned long long)zero_ts);
  }
}

__device__ __forceinline__ void decode_one(int i, int cap, int64_t ts, float val, int slot,
                                           uint64_t trace_h, uint32_t pod, uint32_t pid, uint32_t svcnode,
                                           uint64_t conn_h, const DecodeOut& o, const LdsLane& l,
                                           int& unsupported, int& zero_ts, bool local, void* rec_dst,
                                           uint64_t* t_range = nullptr) {
  uint8_t st = 0;
  if (slot >= 0 && local) {
    const Tables& t = *l.tab;
    st = val >= t.err[slot] ? 2 : (val >= t.warn[slot] ? 1 : 0);
    // bucket = number of finite edges strictly below val ("le" semantics: val <= edge[b])
    const float4* row = reinterpret_cast<const float4*>(t.edges[slot]);
    const float4 r0 = row[0], r1 = row[1], r2 = row[2], r3 = row[3];
    const int b = (val > r0.x) + (val > r0.y) + (val > r0.z) + (val > r0.w) + (val > r1.x) + (val > r1.y) +
                  (val > r1.z) + (val > r1.w) + (val > r2.x) + (val > r2.y) + (val > r2.z) + (val > r2.w) +
                  (val > r3.x) + (val > r3.y) + (val > r3.z);  // r3.w is the +inf overflow edge
    atomicAdd(&l.hist[slot * kBuckets + b], 1u);
    atomicAdd(&l.status[slot * 3 + st], 1u);
    // exact, order-independent integer sum (values are >= 0 by construction)
    const double milli = rint((double)val * 1000.0);
    if (milli > 0.0) atomicAdd(&l.sum[slot], (unsigned long long)milli);
  } else if (slot >= 0) {
    st = val >= l.tab->err[slot] ? 2 : (val >= l.tab->warn[slot] ? 1 : 0);
  } else if (local) {
    ++unsupported;
  }
  o.cols.status[i] = st;
  {
    SigRec r;
    r.ts = ts;
    r.tr = trace_h;
    r.cn = conn_h;
    r.pod = pod;
    r.pid = pid;
    r.sn = svcnode;
    r.val = val;
    r.slot = slot >= 0 ? (uint32_t)slot : kNoSlot;
    // 4 x 16 B: rec_dst is a 64-byte-aligned global row or a 16-byte-aligned LDS staging slot
    const uint4* rs = reinterpret_cast<const uint4*>(&r);
    uint4* rd = static_cast<uint4*>(rec_dst);
#pragma unroll
    for (int q = 0; q < 4; ++q) rd[q] = rs[q];
  }
  // Unsupported signal types never reach Match (REF correlator.go:73-77), and a zero
  // timestamp never satisfies a window (REF dns.go:107-113): no join keys for either.
  const bool joinable = slot >= 0 && ts != 0;
  if (ts == 0 && local) ++zero_ts;
  if (t_range && joinable) {  // the generation's joinable time range (probe pruning)
    t_range[0] = min(t_range[0], ts_image(ts));
    t_range[1] = max(t_range[1], ts_image(ts));
  }
  PartCodes pc;
#pragma unroll
  for (int k = 0; k < kKeyTypes; ++k) {
    const uint64_t h = joinable ? key_hash(k, trace_h, pod, pid, conn_h, svcnode) : 0ull;
    pc.p[k] = h ? (uint16_t)part_of(h) : kNoPart;
    if (h) atomicAdd(&l.part[k * kParts + part_of(h)], 1u);
  }
  o.cols.part[i] = pc;
}

template <int NT>
__global__ __launch_bounds__(NT) void k_decode_events(const Event* __restrict__ ev, const int* __restrict__ n_ptr,
                                                      int cap, DecodeOut o) {
  __shared__ DecodeLds L;
  lds_init<NT>(L);
  const LdsLane l = lds_lane(L);

  const int n = min(*n_ptr, cap);
  // counts[3] = number of node-local events; events past it are imported halo / remote
  // trace-tagged copies that take part in the join but not in the window's counters.
  const int n_local = n_ptr[3] > 0 ? min(n_ptr[3], n) : n;
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);
  int unsupported = 0, zero_ts = 0;
  for (int i = beg + threadIdx.x; i < end; i += NT) {
    const Event e = ev[i];
    const int st = e.signal_type;
    const int slot = st < kMaxTypes ? (int)L.tab.type_slot[st] : -1;
    const float val = slot >= 0 ? (float)((double)e.value * (double)L.tab.scale[slot]) : (float)e.value;
    const uint64_t ch = e.conn_h ? e.conn_h : conn_hash(e.src_port, e.dst_port, e.dst_ip);
    const uint32_t svcnode = ((uint32_t)e.svc_id << 16) | e.node_id;
    decode_one(i, cap, e.ts_ns, val, slot, e.trace_h, e.pod_id, e.pid, svcnode, ch, o, l, unsupported, zero_ts, i < n_local, o.cols.rec + i);
  }
  lds_flush<NT>(L, o, unsupported, zero_ts);
}

// Group sharding (one node's stream split across the node's GPUs, ``agent --gpus N``): every
// GPU decodes the whole window, but only the records of the services it owns (service s >= 1
// -> GPU (s - 1) % world; records of no service -> GPU 0) are counted and joined; the rest
// become holes. Incident group g (service g + 1) lives on GPU g % world as local group g / world.
__device__ __forceinline__ bool shard_owns(uint32_t svcnode, int rank, int world) {
  if (world <= 1) return true;
  const uint32_t svc = svcnode >> 16;
  return (svc ? (int)((svc - 1u) % (uint32_t)world) : 0) == rank;
}

// EVENT16 field accessors: the trace id without its epoch tag; ts = base[tag] + ts_off
__device__ __forceinline__ uint64_t wire_trace(const EventC16& e) { return (uint64_t)(e.trace_id & kTraceIdMask); }
__device__ __forceinline__ int64_t wire_ts(const EventC16& e, const int64_t* base) {
  return e.ts_off == kTsZero ? 0 : base[e.trace_id >> kEpochTagShift] + (int64_t)e.ts_off;
}

// EVENT16 records (the BPF ring's payloads, compacted by the agent's consumer, plus host-encoded
// user-space records). Context rows resolve through the device context table.
template <int NT, class Rec>
__global__ __launch_bounds__(NT) void k_decode_wire(const Rec* __restrict__ ev, const int* __restrict__ n_ptr,
                                                    int cap, const uint4* __restrict__ ctx_tab, int n_ctx,
                                                    DecodeOut o) {
  __shared__ DecodeLds L;
  lds_init<NT>(L);
  const LdsLane l = lds_lane(L);

  const int n = min(*n_ptr, cap);
  const int n_local = n_ptr[3] > 0 ? min(n_ptr[3], n) : n;
  // epoch bases: [0] = counts[4..5] (the window base), [1..3] = counts[8..13]
  auto base_at = [&](int lo) { return (int64_t)(((uint64_t)(uint32_t)n_ptr[lo + 1] << 32) | (uint32_t)n_ptr[lo]); };
  const int64_t t_base[4] = {base_at(4), base_at(8), base_at(10), base_at(12)};
  // counts[6] = rows of the (fixed-capacity, append-only) context table valid this window
  if (n_ptr[6] > 0) n_ctx = min(n_ptr[6], n_ctx);
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);
  int unsupported = 0, zero_ts = 0;
  // software pipeline: the next record and its context row are loaded while this one is
  // decoded (one workgroup per CU at this grid: the loads must overlap the LDS work)
  auto ctx_of = [&](const Rec& r) {
    const uint32_t cid = r.ctx_type >> 8;
    return cid < (uint32_t)n_ctx ? ctx_tab[cid] : make_uint4(0u, 0u, 0u, 0u);
  };
  // Row records leave through LDS: a lane's 64-byte SigRec stored straight to global memory
  // makes every store instruction touch 64 cache lines; staged, each wave writes its 64
  // consecutive records (4 KiB) as 4 fully coalesced 1 KiB stores. Trip counts are uniform
  // across the workgroup (the staging needs barriers).
  // padded to 5 x 16 B per record: at a 64-byte stride the 16-byte stores of a lane group hit
  // the same banks
  __shared__ uint4 s_stage[NT * 5];
  const int lane = threadIdx.x & 63, wbase = threadIdx.x & ~63;
  const int trips = end > beg ? (end - beg + NT - 1) / NT : 0;
  int i = beg + threadIdx.x;
  Rec e_nx{};
  uint4 cx_nx = make_uint4(0u, 0u, 0u, 0u);
  if (i < end) {
    e_nx = ev[i];
    cx_nx = ctx_of(e_nx);
  }
  for (int it = 0; it < trips; ++it, i += NT) {
    const Rec e = e_nx;
    const uint4 cx = cx_nx;
    if (i + NT < end) {
      e_nx = ev[i + NT];
      cx_nx = ctx_of(e_nx);
    }
    if (i < end) {
      const int st = (int)(e.ctx_type & 0xFFu);
      const int slot = st < kMaxTypes ? (int)L.tab.type_slot[st] : -1;
      const float val = (float)((double)e.value_milli * 1e-3);
      const int64_t ts = wire_ts(e, t_base);
      const uint64_t tr = wire_trace(e);
      decode_one(i, cap, ts, val, slot, tr, cx.x, cx.y, cx.w, (uint64_t)cx.z, o, l, unsupported, zero_ts,
                 i < n_local, &s_stage[threadIdx.x * 5]);
    }
    __syncthreads();
    const int first = i - lane;  // this wave's first record
    const int nv = min(64, end - first);
    if (nv > 0) {
      const uint4* src = &s_stage[wbase * 5];
      uint4* dst = reinterpret_cast<uint4*>(o.cols.rec + first);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = lane + 64 * j;  // 16-byte chunk q of the wave's 4 KiB
        if ((q >> 2) < nv) dst[q] = src[(q >> 2) * 5 + (q & 3)];
      }
    }
    __syncthreads();
  }
  lds_flush<NT>(L, o, unsupported, zero_ts);
}

// ---- the native engine's window: BPF ring bytes + user-space records, decoded on the GPU ----

// One pass over the slots of the window's framed batch records (136-byte stride, 8 slots each:
// one thread per slot, the 8 threads of a record share its header line) before the decode:
// applies the probes' id definitions -- context rows into the device context table (svc|node
// from the device pod table), trace id -> hash into the device trace-id table -- and finds the
// first record still being written (a consumer must stop there; the host re-submits the rest
// later). A window holds at most one definition per id (ids are reused only after 2^24 new
// traces or an agent-side context reset), so the stores need no ordering among themselves.
__global__ __launch_bounds__(256) void k_ring_defs(const uint8_t* __restrict__ framed, const int* __restrict__ n_ptr,
                                                   uint4* __restrict__ ctx_tab, uint32_t ctx_rows,
                                                   const uint32_t* __restrict__ pod_sn, uint32_t n_pods, TraceIds tt,
                                                   uint32_t* __restrict__ rs) {
  const int n = n_ptr[15];  // framed rows (slots) in this window
  uint32_t foreign = 0, dctx = 0, dtr = 0, disc = 0, busy = 0xFFFFFFFFu;
  // kU records per thread per trip, all 3 x kU loads issued before any is used: the pass is
  // bound by memory latency, not bytes (a header load followed by a dependent payload load
  // per record ran at ~0.6 TB/s)
  constexpr int kU = 4;
  const int stride = gridDim.x * 256;
  for (int i0 = blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * kU) {
    uint2 h[kU], a[kU], b[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * stride;
      if (i < n) {
        // 8-byte loads: records are 136 bytes apart, so slots are 8- but not 16-byte aligned
        const uint2* sl = reinterpret_cast<const uint2*>(framed + slot_off(i));
        h[u] = *reinterpret_cast<const uint2*>(framed + rec_off(i));
        a[u] = sl[0];
        b[u] = sl[1];
      } else {
        h[u] = make_uint2(kRecPayload, 0u);
        a[u] = b[u] = make_uint2(0u, 0u);
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * stride;
      if (i >= n) continue;
      if (h[u].x & kRbBusy) {
        busy = min(busy, (uint32_t)i);
        continue;
      }
      if ((h[u].x & ~(kRbBusy | kRbDiscard)) != kRecPayload) {
        foreign += (i & 7) == 0;  // once per record
        continue;
      }
      if (h[u].x & kRbDiscard) {
        disc += (i & 7) == 0;
        continue;
      }
      const uint32_t type = a[u].y & 0xFFu;
      if (type == kDefCtx) {  // {conn32, type | id << 8, pod, pid}
        const uint32_t id = a[u].y >> 8;
        if (id && id < ctx_rows) {
          ctx_tab[id] = make_uint4(b[u].x, b[u].y, a[u].x, b[u].x < n_pods ? pod_sn[b[u].x] : 0u);
          ++dctx;
        }
      } else if (type == kDefTrace) {  // {id, type, hash lo, hash hi}
        const unsigned long long hash = (unsigned long long)b[u].x | ((unsigned long long)b[u].y << 32);
        if (hash && a[u].x && a[u].x < tt.n) {
          tt.hash[a[u].x] = hash;
          ++dtr;
        }
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    foreign += __shfl_xor(foreign, off);
    dctx += __shfl_xor(dctx, off);
    dtr += __shfl_xor(dtr, off);
    disc += __shfl_xor(disc, off);
    busy = min(busy, (uint32_t)__shfl_xor((int)busy, off));
  }
  // one global atomic per workgroup and counter: definitions are spread over the whole ring,
  // so nearly every wave has some, and per-wave atomics on the same five L2 addresses
  // serialised (measured: 86 us for a 1M-record window at 4 waves/SIMD, vs ~30 us here)
  __shared__ uint32_t s_acc[5];
  if (threadIdx.x < 5) s_acc[threadIdx.x] = threadIdx.x == 0 ? 0xFFFFFFFFu : 0u;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    if (busy != 0xFFFFFFFFu) atomicMin(&s_acc[0], busy);
    if (foreign) atomicAdd(&s_acc[1], foreign);
    if (dctx) atomicAdd(&s_acc[2], dctx);
    if (dtr) atomicAdd(&s_acc[3], dtr);
    if (disc) atomicAdd(&s_acc[4], disc);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_acc[0] != 0xFFFFFFFFu) atomicMin(&rs[kRsFirstBusy], s_acc[0]);
    if (s_acc[1]) atomicAdd(&rs[kRsForeign], s_acc[1]);
    if (s_acc[2]) atomicAdd(&rs[kRsDefCtx], s_acc[2]);
    if (s_acc[3]) atomicAdd(&rs[kRsDefTrace], s_acc[3]);
    if (s_acc[4]) atomicAdd(&rs[kRsDiscard], s_acc[4]);
  }
}

// Rows [0, counts[15]) come from the slots of the framed batch records (row i = slot i % 8 of
// record i / 8; definitions, pads, discarded, foreign and not-yet-committed records become
// holes: no counters, no join keys),
// rows [counts[15], counts[0]) from the user-space producers' 64-byte EVENT records, whose
// connection keys fold to the conn32 of the context rows (kernel records' trace ids become
// their hashes through the trace-id table; user records carry hashes), so both kinds of record
// join the same spans identically; rows [counts[0], rows[0]) are imported SigRecs (the halo of
// the previous window, other GPUs' trace-tagged records): decoded for the join only.
template <int NT>
__global__ __launch_bounds__(NT) void k_decode_window(const uint8_t* __restrict__ framed,
                                                      const Event* __restrict__ user, const int* __restrict__ n_ptr,
                                                      const int* __restrict__ rows, int cap,
                                                      const SigRec* __restrict__ imp,
                                                      const uint4* __restrict__ ctx_tab, int n_ctx, TraceIds tt,
                                                      uint32_t* __restrict__ rs, unsigned long long* __restrict__ tmax,
                                                      const uint32_t* __restrict__ pod_sn, uint32_t n_pods, int seg,
                                                      int sh_rank, int sh_world, DecodeOut o) {
  __shared__ DecodeLds L;
  // the workgroup's scalar results, merged in LDS first: one global atomic per workgroup and
  // counter (per-wave atomics put 4096 waves x 5 updates per window on the same few L2 lines)
  __shared__ uint32_t s_cnt2[3];
  __shared__ unsigned long long s_t[3];
  if (threadIdx.x == 0) {
    s_cnt2[0] = s_cnt2[1] = s_cnt2[2] = 0u;
    s_t[0] = 0ull;
    s_t[1] = ~0ull;
    s_t[2] = 0ull;
  }
  lds_init<NT>(L);
  const LdsLane l = lds_lane(L);
  // segment 0: rows [0, rows[0]) (the window's records and its halo); segment 1: rows
  // [rows[0], rows[1]) (other GPUs' rows, decoded once they have been all-gathered)
  const int r0 = min(rows[0], cap);
  const int seg_beg = seg ? r0 : 0;
  const int n = seg ? max(r0, min(rows[1], cap)) : r0;
  const int n_loc = min(n_ptr[0], r0);
  const int n_k = min(n_ptr[15], n_loc);
  const int user_rec = n_ptr[6];  // counts[6]: user-space record bytes (64 = EVENT, 32 = User32, 24 = User24, 16 = User16)
  const int valid_k = min((int)min((uint32_t)n_k, rs[kRsFirstBusy]), n_k);
  auto base_at = [&](int lo) { return (int64_t)(((uint64_t)(uint32_t)n_ptr[lo + 1] << 32) | (uint32_t)n_ptr[lo]); };
  const int64_t t_base[4] = {base_at(4), base_at(8), base_at(10), base_at(12)};
  // USER24 timestamps resolve against the newest epoch base (tags rotate; unset bases are 0)
  const int64_t u_base = max(max(t_base[0], t_base[1]), max(t_base[2], t_base[3]));
  const int chunk = (n - seg_beg + gridDim.x - 1) / gridDim.x;
  const int beg = seg_beg + blockIdx.x * chunk, end = min(n, beg + chunk);
  int unsupported = 0, zero_ts = 0, events = 0, other = 0;
  uint32_t n_sel = 0;  // lane 0 of each wave: its selected rows
  unsigned long long t_hi = 0;
  uint64_t tr[2] = {~0ull, 0ull};  // joinable rows' time range (u64 images)
  // rows land in the current generation's slot (resident for the halo)
  const uint32_t cur = cur_slot(o.cols);
  SigRec* const rec_out = o.cols.rec + (size_t)cur * (size_t)o.cols.stride;
  __shared__ uint4 s_stage[NT * 5];
  const int lane = threadIdx.x & 63, wbase = threadIdx.x & ~63;
  const int trips = end > beg ? (end - beg + NT - 1) / NT : 0;
  int i = beg + threadIdx.x;
  for (int it = 0; it < trips; ++it, i += NT) {
    if (i < end) {
      if (i >= n_loc) {  // imported row: joins, never counted
        const SigRec& m = imp[i - n_loc];
        decode_one(i, cap, m.ts, m.val, m.slot == kNoSlot ? -1 : (int)m.slot, m.tr, m.pod, m.pid, m.sn, m.cn, o, l,
                   unsupported, zero_ts, false, &s_stage[threadIdx.x * 5], tr);
      } else if (i < n_k) {  // slot i & 7 of batch record i >> 3
        const uint2 h = *reinterpret_cast<const uint2*>(framed + rec_off(i));
        const uint2* sl = reinterpret_cast<const uint2*>(framed + slot_off(i));
        const uint2 a = sl[0], b = sl[1];
        const EventC16 e{a.x, a.y, b.x, b.y};
        bool ok = i < valid_k && h.x == kRecPayload && (e.ctx_type & 0xFFu) < kDefFirst;
        const uint32_t cid = e.ctx_type >> 8;
        uint4 cx = ok && cid < (uint32_t)n_ctx ? ctx_tab[cid] : make_uint4(0u, 0u, 0u, 0u);
        // the pod's service as the pod table knows it now: a context defined before the pod's
        // first span reached the agent stored svc 0, which would keep its records on GPU 0
        const uint32_t sn_now = cx.x < n_pods ? pod_sn[cx.x] : 0u;
        if (sn_now) cx.w = sn_now;
        if (ok && !shard_owns(cx.w, sh_rank, sh_world)) {
          ok = false;
          ++other;
        }
        if (ok) {
          const int st = (int)(e.ctx_type & 0xFFu);
          const int slot = st < kMaxTypes ? (int)L.tab.type_slot[st] : -1;
          const int64_t ts = wire_ts(e, t_base);
          decode_one(i, cap, ts, (float)((double)e.value_milli * 1e-3), slot, trace_of(tt, (uint32_t)wire_trace(e)),
                     cx.x, cx.y, cx.w, (uint64_t)cx.z, o, l, unsupported, zero_ts, true, &s_stage[threadIdx.x * 5], tr);
          if (slot >= 0 && ts > 0) t_hi = max(t_hi, (unsigned long long)ts);
          ++events;
        } else {  // a hole: never counted, never joined
          decode_one(i, cap, 0, 0.f, -1, 0, 0, 0, 0, 0, o, l, unsupported, zero_ts, false, &s_stage[threadIdx.x * 5], tr);
        }
      } else if (user_rec == 16) {
        const int j = i - n_k;
        const uint4 u = reinterpret_cast<const uint4*>(user)[j];  // {ts_lo, value, pid_sig, pod_ts}
        const uint32_t pod = u.w & 0xFFFFFu;
        const uint32_t sn = pod < n_pods ? pod_sn[pod] : 0u;
        if (u.z == kUser16Cont) {  // a continuation slot: the previous record's trace, not a record
          decode_one(i, cap, 0, 0.f, -1, 0, 0, 0, 0, 0, o, l, unsupported, zero_ts, false, &s_stage[threadIdx.x * 5], tr);
        } else if (!shard_owns(sn, sh_rank, sh_world)) {
          ++other;
          decode_one(i, cap, 0, 0.f, -1, 0, 0, 0, 0, 0, o, l, unsupported, zero_ts, false, &s_stage[threadIdx.x * 5], tr);
        } else {
          uint64_t trh = 0;
          if ((u.z & kUser16Trace) && i + 1 < n_loc) {
            const uint4 c = reinterpret_cast<const uint4*>(user)[j + 1];
            if (c.z == kUser16Cont) trh = ((uint64_t)c.y << 32) | c.x;
          }
          const uint32_t ps = u.z & ~kUser16Trace;
          const int st = (int)((ps >> 22) & 0x7Fu);
          const int slot = (int)L.tab.type_slot[st];
          const int64_t ts = user24_ts(u.x, u.w, ps, u_base);
          decode_one(i, cap, ts, (float)((double)u.y * 1e-3), slot, trh, pod, ps & 0x3FFFFFu, sn, 0ull, o, l,
                     unsupported, zero_ts, true, &s_stage[threadIdx.x * 5], tr);
          if (slot >= 0 && ts > 0) t_hi = max(t_hi, (unsigned long long)ts);
          ++events;
        }
      } else if (user_rec == 24) {
        const uint2* u = reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(user) + (size_t)(i - n_k) * 24);
        const uint2 a = u[0], b = u[1], c = u[2];  // {trace lo, hi}, {value, ts_lo}, {pid_sig, pod_ts}
        const int st = (int)((c.x >> 22) & 0x7Fu);
        const int slot = (int)L.tab.type_slot[st];
        const uint32_t pod = c.y & 0xFFFFFu;
        const uint32_t sn = pod < n_pods ? pod_sn[pod] : 0u;
        const int64_t ts = user24_ts(b.y, c.y, c.x, u_base);
        if (!shard_owns(sn, sh_rank, sh_world)) {
          ++other;
          decode_one(i, cap, 0, 0.f, -1, 0, 0, 0, 0, 0, o, l, unsupported, zero_ts, false, &s_stage[threadIdx.x * 5], tr);
        } else {
        decode_one(i, cap, ts, (float)((double)b.x * 1e-3), slot, ((uint64_t)a.y << 32) | a.x, pod, c.x & 0x3FFFFFu, sn,
                   0ull, o, l, unsupported, zero_ts, true, &s_stage[threadIdx.x * 5], tr);
        if (slot >= 0 && ts > 0) t_hi = max(t_hi, (unsigned long long)ts);
        ++events;
        }
      } else if (user_rec == 32) {
        const User32 e = reinterpret_cast<const User32*>(user)[i - n_k];
        const int st = e.signal_type;
        const int slot = st < kMaxTypes ? (int)L.tab.type_slot[st] : -1;
        const uint32_t sn = e.pod_id < n_pods ? pod_sn[e.pod_id] : 0u;
        if (!shard_owns(sn, sh_rank, sh_world)) {
          ++other;
          decode_one(i, cap, 0, 0.f, -1, 0, 0, 0, 0, 0, o, l, unsupported, zero_ts, false, &s_stage[threadIdx.x * 5], tr);
        } else {
        decode_one(i, cap, e.ts_ns, (float)((double)e.value_milli * 1e-3), slot, e.trace_h, e.pod_id, e.pid, sn, 0ull,
                   o, l, unsupported, zero_ts, true, &s_stage[threadIdx.x * 5], tr);
        if (slot >= 0 && e.ts_ns > 0) t_hi = max(t_hi, (unsigned long long)e.ts_ns);
        ++events;
        }
      } else {
        const Event e = user[i - n_k];
        const int st = e.signal_type;
        const int slot = st < kMaxTypes ? (int)L.tab.type_slot[st] : -1;
        const float val = slot >= 0 ? (float)((double)e.value * (double)L.tab.scale[slot]) : (float)e.value;
        const uint64_t ck = e.conn_h ? e.conn_h : conn_hash(e.src_port, e.dst_port, e.dst_ip);
        const uint32_t svcnode = ((uint32_t)e.svc_id << 16) | e.node_id;
        if (!shard_owns(svcnode, sh_rank, sh_world)) {
          ++other;
          decode_one(i, cap, 0, 0.f, -1, 0, 0, 0, 0, 0, o, l, unsupported, zero_ts, false, &s_stage[threadIdx.x * 5], tr);
        } else {
          decode_one(i, cap, e.ts_ns, val, slot, e.trace_h, e.pod_id, e.pid, svcnode, conn32(ck), o, l, unsupported,
                     zero_ts, true, &s_stage[threadIdx.x * 5], tr);
          if (slot >= 0 && e.ts_ns > 0) t_hi = max(t_hi, (unsigned long long)e.ts_ns);
          ++events;
        }
      }
    }
    __syncthreads();
    if (o.sel_mask) {  // a warn-level (or worse) trace-tagged joinable local row (exchange.hip selected())
      bool sel = false;
      if (i < end && i < n_loc) {
        const SigRec& r = *reinterpret_cast<const SigRec*>(&s_stage[threadIdx.x * 5]);
        sel = r.slot != kNoSlot && r.ts != 0 && r.tr != 0 && (r.val >= L.tab.err[r.slot] || r.val >= L.tab.warn[r.slot]);
      }
      const unsigned long long m = __ballot(sel);
      if (lane == 0) {
        o.sel_mask[(size_t)blockIdx.x * o.sel_stride + (size_t)it * (NT / 64) + (threadIdx.x >> 6)] = m;
        n_sel += (uint32_t)__popcll(m);
      }
    }
    const int first = i - lane;
    const int nv = min(64, end - first);
    if (nv > 0) {
      const uint4* src = &s_stage[wbase * 5];
      uint4* dst = reinterpret_cast<uint4*>(rec_out + first);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = lane + 64 * j;
        if ((q >> 2) < nv) dst[q] = src[(q >> 2) * 5 + (q & 3)];
      }
    }
    __syncthreads();
  }
  for (int off = 32; off > 0; off >>= 1) {
    events += __shfl_xor(events, off);
    other += __shfl_xor(other, off);
    t_hi = max(t_hi, (unsigned long long)__shfl_xor((long long)t_hi, off));
    tr[0] = min(tr[0], (uint64_t)__shfl_xor((long long)tr[0], off));
    tr[1] = max(tr[1], (uint64_t)__shfl_xor((long long)tr[1], off));
  }
  if ((threadIdx.x & 63) == 0) {
    if (events) atomicAdd(&s_cnt2[0], (uint32_t)events);
    if (other) atomicAdd(&s_cnt2[1], (uint32_t)other);
    if (n_sel) atomicAdd(&s_cnt2[2], n_sel);
    if (t_hi) atomicMax(&s_t[0], t_hi);
    if (tr[0] <= tr[1]) {
      atomicMin(&s_t[1], (unsigned long long)tr[0]);
      atomicMax(&s_t[2], (unsigned long long)tr[1]);
    }
  }
  lds_flush<NT>(L, o, unsupported, zero_ts);  // starts with a barrier: s_cnt2 / s_t are final
  if (threadIdx.x == 0) {
    if (s_cnt2[0]) atomicAdd(&rs[kRsEvents], s_cnt2[0]);
    if (s_cnt2[1]) atomicAdd(&rs[kRsOtherShard], s_cnt2[1]);
    if (o.sel_cnt) o.sel_cnt[blockIdx.x] = s_cnt2[2];  // every block, zero included (the scan reads all)
    if (s_t[0]) atomicMax(tmax, s_t[0]);
    if (o.cols.gen && s_t[1] <= s_t[2]) {
      atomicMin(reinterpret_cast<unsigned long long*>(&o.cols.gen->tlo[cur]), s_t[1]);
      atomicMax(reinterpret_cast<unsigned long long*>(&o.cols.gen->thi[cur]), s_t[2]);
    }
  }
}

// REF 40-byte records: REF units (count stays count, cpu_steal raw ns, else ns/1e6) and
// workload identity supplied by the consumer (REF EventMetadata, ringbuf.go:19-26).
template <int NT>
__global__ __launch_bounds__(NT) void k_decode_ref(const RefEvent* __restrict__ ev, const int* __restrict__ n_ptr,
                                                   int cap, uint32_t pod, uint32_t svcnode, uint64_t trace_h,
                                                   DecodeOut o) {
  __shared__ DecodeLds L;
  lds_init<NT>(L);
  const LdsLane l = lds_lane(L);
  const int n = min(*n_ptr, cap);
  // counts[3] = number of node-local events; events past it are imported halo / remote
  // trace-tagged copies that take part in the join but not in the window's counters.
  const int n_local = n_ptr[3] > 0 ? min(n_ptr[3], n) : n;
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);
  int unsupported = 0, zero_ts = 0;
  for (int i = beg + threadIdx.x; i < end; i += NT) {
    const RefEvent e = ev[i];
    const uint32_t st = e.signal_type;
    int slot = (st >= 1 && st <= 9) ? (int)L.tab.type_slot[st] : -1;
    float val;
    if (st == 2 || st == 6) val = (float)e.value_ns;           // tcp count, cpu_steal raw ns
    else val = (float)((double)e.value_ns / 1e6);               // ns -> ms
    const uint64_t ch = conn_hash(e.conn_src_port, e.conn_dst_port, e.conn_dst_ip);
    decode_one(i, cap, (int64_t)e.timestamp_ns, val, slot, trace_h, pod, e.pid, svcnode, ch, o, l, unsupported, zero_ts, i < n_local, o.cols.rec + i);
  }
  lds_flush<NT>(L, o, unsupported, zero_ts);
}

// Span records -> span columns + span partition counts. n_ptr = counts + 1: n_ptr[0] spans,
// n_ptr[5] valid context rows, n_ptr[6] span record bytes (20 = SpanC20 via the context table).
constexpr int kSliLds = 1024;  // groups whose SLO counts k_decode_spans keeps in LDS

template <int NT>
__global__ __launch_bounds__(NT) void k_decode_spans(const void* __restrict__ sp_raw, const int* __restrict__ n_ptr,
                                                     int cap, SpanCols c, uint32_t* part_cnt,
                                                     const uint4* __restrict__ ctx_tab, int n_ctx, SpanMap sm) {
  const Span* __restrict__ sp = static_cast<const Span*>(sp_raw);
  const SpanC20* __restrict__ sp20 = static_cast<const SpanC20*>(sp_raw);
  const bool compact = n_ptr[6] == 20;
  if (n_ptr[5] > 0) n_ctx = min(n_ptr[5], n_ctx);
  __shared__ uint32_t s_part[kKeyTypes * kParts];
  // per-incident SLO counts privatised in LDS: a window's spans all land on its few groups, so
  // global atomics serialised on a handful of L2 addresses (33 us per 16K-span window)
  __shared__ uint32_t s_sli[2 * kSliLds];
  __shared__ uint32_t s_app[2 * kSliLds];  // application retrieval: spans, sum (10 us units)
  __shared__ uint32_t s_late[kSliLds];     // late breaches
  const bool sli_lds = sm.grp_sli && sm.n_groups <= kSliLds;
  const bool app_lds = sm.grp_app && sm.n_groups <= kSliLds;
  for (int i = threadIdx.x; i < kKeyTypes * kParts; i += NT) s_part[i] = 0;
  if (sli_lds)
    for (int i = threadIdx.x; i < 2 * sm.n_groups; i += NT) s_sli[i] = 0;
  if (app_lds)
    for (int i = threadIdx.x; i < 2 * sm.n_groups; i += NT) s_app[i] = 0;
  const bool late_lds = sm.grp_late && sm.n_groups <= kSliLds;
  if (late_lds)
    for (int i = threadIdx.x; i < sm.n_groups; i += NT) s_late[i] = 0;
  __syncthreads();
  const int n = min(*n_ptr, cap);
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);
  uint64_t t_lo = ~0ull, t_hi = 0ull;  // joinable spans' time range (u64 images)
  for (int i = beg + threadIdx.x; i < end; i += NT) {
    SpanRec r;
    if (compact) {
      const SpanC20 s = sp20[i];
      const uint4 cx = s.ctx_id < (uint32_t)n_ctx ? ctx_tab[s.ctx_id] : make_uint4(0u, 0u, 0u, 0u);
      r.ts = s.ts_ns;
      r.tr = s.trace_id;
      r.cn = cx.z;
      r.pod = cx.x;
      r.pid = cx.y;
      r.sn = cx.w;
      r.grp = s.group_id;
      if (sm.sh_world > 1) {  // another GPU's incident group: a span row that never joins
        if (r.grp % (uint32_t)sm.sh_world != (uint32_t)sm.sh_rank) r.ts = 0;
        r.grp /= (uint32_t)sm.sh_world;
      }
    } else {
      const Span s = sp[i];
      r.ts = s.ts_ns;
      // native engine: connections as conn32 (the context rows' identity); trace hashes as is
      r.tr = s.trace_h;
      r.cn = sm.native ? (uint64_t)conn32(s.conn_h) : s.conn_h;
      uint32_t grp = s.group_id;
      bool mine = true;
      if (sm.sh_world > 1) {
        mine = grp % (uint32_t)sm.sh_world == (uint32_t)sm.sh_rank;
        grp /= (uint32_t)sm.sh_world;
        if (!mine) r.ts = 0;  // another GPU's incident group: never joins, never counted here
      }
      // a first-token record (kSpanFirstToken) joins like its request span: the request's evidence
      // reaches the window its SLI is counted in, not the one its request span is exported in
      // per-incident TTFT SLO accounting (a request whose first-token record counted it: once)
      if (mine && sm.grp_sli && grp < (uint32_t)sm.n_groups && !(s.flags & kSpanNoSli)) {
        const bool breach = s.ttft_ms > sm.ttft_slo_ms;
        if (breach && (s.flags & kSpanLate) && sm.grp_late) {  // an earlier window's breach, reported now
          if (late_lds) atomicAdd(&s_late[grp], 1u);
          else atomicAdd(&sm.grp_late[2 * grp], 1u);
        } else {
          uint32_t* sli = sli_lds ? s_sli : sm.grp_sli;
          atomicAdd(&sli[2 * grp], 1u);
          if (breach) atomicAdd(&sli[2 * grp + 1], 1u);
        }
      }
      // the application's retrieval time of the request (REF DecomposeRetrieval's input,
      // correlator.go:179-194): its group sum, in fixed point like every incident sum
      if (mine && sm.grp_app && grp < (uint32_t)sm.n_groups && s.retr_ms > 0.f && s.retr_ms < 1e7f) {
        uint32_t* app = app_lds ? s_app : sm.grp_app;
        atomicAdd(&app[2 * grp], 1u);
        atomicAdd(&app[2 * grp + 1], (uint32_t)rint((double)s.retr_ms * kAppUnitsPerMs));
      }
      r.pod = s.pod_id;
      r.pid = s.pid;
      r.sn = ((uint32_t)s.svc_id << 16) | s.node_id;
      r.grp = grp;
    }
    c.rec[i] = r;
    if (r.ts != 0) {
      t_lo = min(t_lo, ts_image(r.ts));
      t_hi = max(t_hi, ts_image(r.ts));
    }
    PartCodes pc;
#pragma unroll
    for (int k = 0; k < kKeyTypes; ++k) {
      const uint64_t h = r.ts != 0 ? key_hash(k, r.tr, r.pod, r.pid, r.cn, r.sn) : 0ull;
      pc.p[k] = h ? (uint16_t)part_of(h) : kNoPart;
      if (h) atomicAdd(&s_part[k * kParts + part_of(h)], 1u);
    }
    c.part[i] = pc;
  }
  if (sm.gen) {
    for (int off = 32; off > 0; off >>= 1) {
      t_lo = min(t_lo, (uint64_t)__shfl_xor((long long)t_lo, off));
      t_hi = max(t_hi, (uint64_t)__shfl_xor((long long)t_hi, off));
    }
    if ((threadIdx.x & 63) == 0 && t_lo <= t_hi) {
      atomicMin(reinterpret_cast<unsigned long long*>(&sm.gen->span_lo), (unsigned long long)t_lo);
      atomicMax(reinterpret_cast<unsigned long long*>(&sm.gen->span_hi), (unsigned long long)t_hi);
    }
  }
  __syncthreads();
  store_counts<NT>(s_part, part_cnt + (size_t)blockIdx.x * kKeyTypes * kParts);
  if (sli_lds)
    for (int i = threadIdx.x; i < 2 * sm.n_groups; i += NT)
      if (s_sli[i]) atomicAdd(&sm.grp_sli[i], s_sli[i]);
  if (app_lds)
    for (int i = threadIdx.x; i < 2 * sm.n_groups; i += NT)
      if (s_app[i]) atomicAdd(&sm.grp_app[i], s_app[i]);
  if (late_lds)
    for (int i = threadIdx.x; i < sm.n_groups; i += NT)
      if (s_late[i]) atomicAdd(&sm.grp_late[2 * i], s_late[i]);
}

// Event decoders run 1024 threads per workgroup: the grid is capped at kPartBlocks (the
// per-block partition matrix the scan consumes), so a fixed grid of 256 workgroups x 4 waves
// left one wave per SIMD, latency-bound on the record loads; 16 waves per CU hide them.
constexpr int kDecodeNT = 1024;

int decode_sel_stride(int cap) {
  const long long g = decode_grid(cap), chunk = ((long long)cap + g - 1) / g;
  return (int)((chunk + kDecodeNT - 1) / kDecodeNT) * (kDecodeNT / 64);
}

int decode_grid(int cap) {
  // Fixed per-capacity grid (graph-replayable): ~4 events per thread, capped at kPartBlocks.
  long long g = ((long long)cap + 1023) / 1024;
  if (g < 1) g = 1;
  if (g > kPartBlocks) g = kPartBlocks;
  return (int)g;
}

void set_tables(const Tables* host_tables) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_tab), host_tables, sizeof(Tables), 0, hipMemcpyHostToDevice);
}

void launch_decode_events(const void* ev, const int* n_dev, int cap, const SignalCols& cols, uint32_t* hist,
                          uint32_t* status_cnt, uint32_t* part_cnt, unsigned long long* misc, hipStream_t stream) {
  DecodeOut o{cols, hist, status_cnt, part_cnt, misc};
  constexpr int NT = kDecodeNT;
  hipLaunchKernelGGL((k_decode_events<NT>), dim3(decode_grid(cap)), dim3(NT), 0, stream,
                     (const Event*)ev, n_dev, cap, o);
}

void launch_decode_wire(const void* ev, const int* n_dev, int cap, const uint32_t* ctx_tab, int n_ctx,
                        const SignalCols& cols, uint32_t* hist, uint32_t* status_cnt, uint32_t* part_cnt,
                        unsigned long long* misc, hipStream_t stream) {
  DecodeOut o{cols, hist, status_cnt, part_cnt, misc};
  constexpr int NT = kDecodeNT;
  hipLaunchKernelGGL((k_decode_wire<NT, EventC16>), dim3(decode_grid(cap)), dim3(NT), 0, stream,
                     (const EventC16*)ev, n_dev, cap, reinterpret_cast<const uint4*>(ctx_tab), n_ctx, o);
}

void launch_decode_ref(const void* ev, const int* n_dev, int cap, uint32_t pod, uint32_t svcnode, uint64_t trace_h,
                       const SignalCols& cols, uint32_t* hist, uint32_t* status_cnt, uint32_t* part_cnt,
                       unsigned long long* misc, hipStream_t stream) {
  DecodeOut o{cols, hist, status_cnt, part_cnt, misc};
  constexpr int NT = kDecodeNT;
  hipLaunchKernelGGL((k_decode_ref<NT>), dim3(decode_grid(cap)), dim3(NT), 0, stream,
                     (const RefEvent*)ev, n_dev, cap, pod, svcnode, trace_h, o);
}

void launch_decode_spans(const void* sp, const int* n_dev, int cap, const SpanCols& cols, uint32_t* part_cnt,
                         const uint32_t* ctx_tab, int n_ctx, hipStream_t stream, const SpanMap* sm) {
  constexpr int NT = 1024;  // the grid is decode_grid(cap) (the span partition matrix): ~1 span per thread
  SpanMap m{};
  if (sm) m = *sm;
  hipLaunchKernelGGL((k_decode_spans<NT>), dim3(decode_grid(cap)), dim3(NT), 0, stream, sp, n_dev, cap, cols,
                     part_cnt, reinterpret_cast<const uint4*>(ctx_tab), n_ctx, m);
}

void launch_ring_defs(const uint8_t* framed, const int* n_dev, int cap, uint32_t* ctx_tab, uint32_t ctx_rows,
                      const uint32_t* pod_sn, uint32_t n_pods, const TraceIds& tt, uint32_t* ring_state,
                      hipStream_t stream) {
  // ~4 records per thread: the pass is latency-bound (PMC: 94 % of wave time waiting with 2
  // waves per SIMD at 8 records per thread)
  int g = (cap + 1023) / 1024;
  g = g < 1 ? 1 : (g > 2048 ? 2048 : g);
  hipLaunchKernelGGL(k_ring_defs, dim3(g), dim3(256), 0, stream, framed, n_dev, reinterpret_cast<uint4*>(ctx_tab),
                     ctx_rows, pod_sn, n_pods, tt, ring_state);
}

void launch_decode_window(const uint8_t* framed, const void* user, const int* n_dev, const int* rows, int cap,
                          const SigRec* imp, const uint32_t* ctx_tab, int n_ctx, const TraceIds& tt,
                          uint32_t* ring_state, unsigned long long* tmax, const uint32_t* pod_sn, uint32_t n_pods,
                          const SignalCols& cols, uint32_t* hist, uint32_t* status_cnt, uint32_t* part_cnt,
                          unsigned long long* misc, hipStream_t stream, int seg, int grid, int blk_base, int sh_rank,
                          int sh_world, uint32_t* sel_cnt, unsigned long long* sel_mask, int sel_stride) {
  // the fused exchange selection (sel_mask) is scattered by k_sel_scatter_mask with
  // decode_grid(cap) blocks and decode_sel_stride(cap) masks per block: the decode that writes the
  // masks must run that very geometry
  if (sel_mask != nullptr && (grid != 0 || sel_stride != decode_sel_stride(cap)))
    throw std::invalid_argument("launch_decode_window: the fused selection needs the default decode grid");
  DecodeOut o{cols, hist, status_cnt, part_cnt, misc, blk_base, sel_cnt, sel_mask, sel_stride};
  constexpr int NT = kDecodeNT;
  hipLaunchKernelGGL((k_decode_window<NT>), dim3(grid > 0 ? grid : decode_grid(cap)), dim3(NT), 0, stream, framed,
                     (const Event*)user, n_dev, rows, cap, imp, reinterpret_cast<const uint4*>(ctx_tab), n_ctx, tt,
                     ring_state, tmax, pod_sn, n_pods, seg, sh_rank, sh_world, o);
}

}  // namespace mislo
