// K2: radix-partitioned, LDS-staged span <-> signal hash join with REF's 4-tier rules.
//
// REF semantics (pkg/correlation/dns.go:50-113, ebpfcorrelator/correlator.go:50-125):
// a (span, signal) pair matches at the FIRST tier it satisfies -- trace_id exact (1.0),
// pod+pid within 100 ms (0.9), pod+conn within 250 ms (0.8), service+node within 500 ms
// (0.65) -- all inside the outer window, windows compared as |dt| <= w on int64 ns,
// zero timestamps never match. Per span the matches with conf >= threshold are ranked by
// (conf desc, |dt| asc, input order), the best `fanout` (3) are kept and max-merged into
// the span's attribute row; unmatched / low-confidence / fanout-dropped / unsupported
// pairs are counted (DebugStats).
//
// GPU design (MI355X):
//   1. decode (decode.hip) hashes every record's 4 join keys; the top kPartBits hash bits
//      pick one of kParts partitions per key type, counted per workgroup;
//   2. k_part_scan / k_base_scan turn per-workgroup counts into scatter offsets;
//   3. k_scatter writes record indices into partition lists (no global atomics);
//   4. k_probe: one workgroup per (key type, partition) stages the partition's SPANS in
//      LDS (bitonic-sorted by (key hash, ts)), then streams the partition's SIGNALS
//      through it: binary search the key range, walk the |dt| window, drop pairs that
//      satisfy a higher-precedence tier (each pair is found exactly once, at its own
//      tier), and insert accepted candidates into the span's top-3 with a lock-free
//      cascade of 64-bit atomicMin (key = tier | |dt| | signal index, so the numeric
//      minimum IS REF's stable-sort order). The broad service+node tier, which REF can
//      only ever count as low-confidence at the default threshold (0.65 < 0.7), is
//      counted with two binary searches instead of enumerating O(S x N) pairs; pairs of
//      higher tiers that also satisfy it are subtracted (overlap) to keep counts exact.
//   5. k_finalize max-merges the kept candidates per span, writes the confidence and the
//      retrieval decomposition. Incident-group features are the mean value per signal
//      slot over either every accepted candidate pair (group_mode 1, accumulated in the
//      probe) or the spans' merged top-3 attributes (group_mode 0, REF-style).
#include <cstdlib>

#include "mislo_common.h"
#include "mislo_launch.h"

namespace mislo {

constexpr int kSigBits = 27;  // top-3 key: [63:62] tier, [61:27] |dt| ns, [26:0] signal idx
constexpr int kChunk = 256;   // spans staged in LDS per pass

// ---------------------------------------------------------------------------------------
// partition scan + scatter
// ---------------------------------------------------------------------------------------

// part_blk[b][c] counts -> part_off[b][c] exclusive prefix over blocks, part_tot[c].
// A column scan over the [nblk][4096] matrix. One thread per column left 64 waves on the
// whole chip, each walking 256 dependent rows; here a workgroup owns kScanCols columns and
// splits the rows into kScanRG groups: pass 1 sums each group (independent loads, 32 rows
// of a wave read 128 contiguous bytes each), the group prefixes go through LDS, pass 2
// rewrites the group's rows as running offsets.
constexpr int kScanCols = 32, kScanRG = 32;
__global__ __launch_bounds__(kScanCols * kScanRG) void k_part_scan(const uint32_t* __restrict__ part_blk, int nblk,
                                                                  uint32_t* __restrict__ part_off,
                                                                  uint32_t* __restrict__ part_tot) {
  __shared__ uint32_t s_sum[kScanRG][kScanCols];
  const int cl = threadIdx.x % kScanCols, r = threadIdx.x / kScanCols;
  const int c = blockIdx.x * kScanCols + cl;
  const int per = (nblk + kScanRG - 1) / kScanRG;
  const int b0 = min(nblk, r * per), b1 = min(nblk, b0 + per);
  constexpr size_t W = (size_t)kKeyTypes * kParts;
  uint32_t sum = 0;
  for (int b = b0; b < b1; ++b) sum += part_blk[(size_t)b * W + c];
  s_sum[r][cl] = sum;
  __syncthreads();
  uint32_t run = 0, tot = 0;
  for (int q = 0; q < kScanRG; ++q) {
    const uint32_t v = s_sum[q][cl];
    run += q < r ? v : 0u;
    tot += v;
  }
  for (int b = b0; b < b1; ++b) {
    const size_t idx = (size_t)b * W + c;
    const uint32_t v = part_blk[idx];
    part_off[idx] = run;
    run += v;
  }
  if (r == 0) part_tot[c] = tot;
}

// exclusive scan of the kKeyTypes x kParts partition totals (one workgroup, 4 per thread)
// (signals: into the current generation's offsets). A launch of its own: folding it into the
// last k_part_scan workgroup needs a device-scope release per workgroup, which on this GPU
// writes back the XCD's L2 -- measured 89 us for the two fused scans against 25 us unfused
// (profiles/r3_kernels/step4_tried.md).
constexpr int kBaseNT = kKeyTypes * kParts / 4;
__global__ __launch_bounds__(kBaseNT) void k_base_scan(const uint32_t* __restrict__ tot, uint32_t* __restrict__ base,
                                                      const GenMeta* __restrict__ gen) {
  if (gen) base += (size_t)gen->cur * kBaseLen;
  __shared__ uint32_t s[kBaseNT];
  const int t = threadIdx.x;
  uint32_t v[4];
  uint32_t sum = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = tot[t * 4 + j];
    sum += v[j];
  }
  s[t] = sum;
  __syncthreads();
  for (int off = 1; off < kBaseNT; off <<= 1) {
    uint32_t x = t >= off ? s[t - off] : 0;
    __syncthreads();
    s[t] += x;
    __syncthreads();
  }
  uint32_t run = s[t] - sum;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    base[t * 4 + j] = run;
    run += v[j];
  }
  if (t == kBaseNT - 1) base[kKeyTypes * kParts] = s[kBaseNT - 1];
}

template <int NT>
__global__ __launch_bounds__(NT) void k_scatter(const PartCodes* __restrict__ codes, const int* __restrict__ n_ptr,
                                                int cap, const uint32_t* __restrict__ part_off,
                                                const uint32_t* __restrict__ base, uint32_t* __restrict__ items,
                                                int nblk_a) {
  // this workgroup's next slot in every list (list base + the workgroup's offset), bumped by an
  // LDS atomic per entry: two dependent global loads per entry less
  __shared__ uint32_t s_pos[kKeyTypes * kParts];
  {
    const uint32_t* my_off = part_off + (size_t)blockIdx.x * kKeyTypes * kParts;
    for (int i = threadIdx.x; i < kKeyTypes * kParts; i += NT) s_pos[i] = base[i] + my_off[i];
  }
  __syncthreads();
  // the same row ranges the decode blocks had: one segment, or two (nblk_a blocks over
  // [0, n_ptr[0]), the rest over [n_ptr[0], n_ptr[1]))
  const int n0 = min(n_ptr[0], cap);
  const bool two = nblk_a < (int)gridDim.x;
  const bool second = two && (int)blockIdx.x >= nblk_a;
  const int s_beg = second ? n0 : 0;
  const int s_end = second ? max(n0, min(n_ptr[1], cap)) : n0;
  const int g = two ? (second ? (int)gridDim.x - nblk_a : nblk_a) : (int)gridDim.x;
  const int bi = second ? (int)blockIdx.x - nblk_a : (int)blockIdx.x;
  const int chunk = (s_end - s_beg + g - 1) / g;
  const int beg = s_beg + bi * chunk, end = min(s_end, beg + chunk);
  for (int i = beg + threadIdx.x; i < end; i += NT) {
    const PartCodes pc = codes[i];
#pragma unroll
    for (int k = 0; k < kKeyTypes; ++k) {
      if (pc.p[k] == kNoPart) continue;
      items[atomicAdd(&s_pos[k * kParts + pc.p[k]], 1u)] = (uint32_t)i;
    }
  }
}

// Signal scatter: the current generation's partition lists, each entry a row index plus the
// row's (key hash, ts) for the list's key type, written once and streamed by the probe of this
// window and of the later windows the rows stay in the halo for. The hashes are recomputed from
// the row records (the decode kept only their partitions); the rows are read in order.
// (body: block `bid` of `nblk` scatter blocks; `s_pos` = kKeyTypes * kParts words of LDS)
template <int NT>
__device__ __forceinline__ void scatter_sig_body(const SignalCols& gc, const int* __restrict__ n_ptr, int cap,
                                                 const uint32_t* __restrict__ part_off, int nblk_a, int bid,
                                                 int nblk, uint32_t* s_pos) {
  const uint32_t cur = cur_slot(gc);
  const SigRec* rec = gc.rec + (size_t)cur * (size_t)gc.stride;
  const uint32_t* base = gc.base + (size_t)cur * kBaseLen;
  uint32_t* items = gc.items + (size_t)cur * kKeyTypes * (size_t)gc.stride;
  KeyTs* keys = gc.keys + (size_t)cur * kKeyTypes * (size_t)gc.stride;
  // next slot per list (see k_scatter)
  {
    const uint32_t* my_off = part_off + (size_t)bid * kKeyTypes * kParts;
    for (int i = threadIdx.x; i < kKeyTypes * kParts; i += NT) s_pos[i] = base[i] + my_off[i];
  }
  __syncthreads();
  // the row ranges of the decode blocks (see k_scatter)
  const int n0 = min(n_ptr[0], cap);
  const bool two = nblk_a < nblk;
  const bool second = two && bid >= nblk_a;
  const int s_beg = second ? n0 : 0;
  const int s_end = second ? max(n0, min(n_ptr[1], cap)) : n0;
  const int g = two ? (second ? nblk - nblk_a : nblk_a) : nblk;
  const int bi = second ? bid - nblk_a : bid;
  const int chunk = (s_end - s_beg + g - 1) / g;
  const int beg = s_beg + bi * chunk, end = min(s_end, beg + chunk);
  // kU rows per thread per trip, every load of the trip issued before the first is used: the
  // list stores of a row may alias the next row's loads for the compiler, so a row-at-a-time loop
  // waited out one memory latency per row
  constexpr int kU = 4;
  const PartCodes* __restrict__ part = gc.part;
  for (int i0 = beg + threadIdx.x; i0 < end; i0 += NT * kU) {
    PartCodes pc[kU];
    uint4 a[kU], b[kU], c4[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * NT;
      if (i < end) {
        pc[u] = part[i];
        const uint4* v = reinterpret_cast<const uint4*>(rec + i);
        a[u] = v[0];
        b[u] = v[1];
        c4[u] = v[2];
      } else {
        pc[u].p[0] = pc[u].p[1] = pc[u].p[2] = pc[u].p[3] = kNoPart;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if ((pc[u].p[0] & pc[u].p[1] & pc[u].p[2] & pc[u].p[3]) == kNoPart) continue;  // not joinable
      const int64_t ts = (int64_t)(((uint64_t)a[u].y << 32) | a[u].x);
      const uint64_t tr = ((uint64_t)a[u].w << 32) | a[u].z, cn = ((uint64_t)b[u].y << 32) | b[u].x;
#pragma unroll
      for (int k = 0; k < kKeyTypes; ++k) {
        if (pc[u].p[k] == kNoPart) continue;
        const uint32_t pos = atomicAdd(&s_pos[k * kParts + pc[u].p[k]], 1u);
        items[pos] = (uint32_t)(i0 + u * NT);
        keys[pos] = KeyTs{key_hash(k, tr, b[u].z, b[u].w, cn, c4[u].x), ts};
      }
    }
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_scatter_sig(SignalCols gc, const int* __restrict__ n_ptr, int cap,
                                                    const uint32_t* __restrict__ part_off, int nblk_a) {
  __shared__ uint32_t s_pos[kKeyTypes * kParts];
  scatter_sig_body<NT>(gc, n_ptr, cap, part_off, nblk_a, (int)blockIdx.x, (int)gridDim.x, s_pos);
}

// ---------------------------------------------------------------------------------------
// probe
// ---------------------------------------------------------------------------------------

__device__ __forceinline__ bool less_ht(uint64_t h1, int64_t t1, uint64_t h2, int64_t t2) {
  return h1 < h2 || (h1 == h2 && t1 < t2);
}

__device__ __forceinline__ void top3_insert(unsigned long long* slot3, unsigned long long key) {
  // Concurrent insertion into a sorted 3-slot array: each atomicMin keeps the smaller of
  // (slot, key) in the slot and the larger continues down; the multiset is preserved and
  // every slot only decreases, so the final slots are the 3 smallest keys in order.
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const unsigned long long old = atomicMin(slot3 + j, key);
    if (old == kEmpty) return;
    key = old > key ? old : key;
  }
}

__device__ __forceinline__ int64_t iabs64(int64_t x) { return x < 0 ? -x : x; }

// The first 48 bytes of a SigRec (every field the probe reads; the padding is never loaded):
// three 16-byte loads per gathered signal.
struct SigHot {
  int64_t ts;
  uint64_t tr, cn;
  uint32_t pod, pid, sn;
  float val;
  uint32_t slot;
};
__device__ __forceinline__ SigHot load_hot(const SigRec* p) {
  const uint4* v = reinterpret_cast<const uint4*>(p);
  const uint4 a = v[0], b = v[1], c = v[2];
  SigHot h;
  h.ts = (int64_t)(((uint64_t)a.y << 32) | a.x);
  h.tr = ((uint64_t)a.w << 32) | a.z;
  h.cn = ((uint64_t)b.y << 32) | b.x;
  h.pod = b.z;
  h.pid = b.w;
  h.sn = c.x;
  h.val = __uint_as_float(c.y);
  h.slot = c.z;
  return h;
}

// Work decomposition: two launches (the trace tier first, then pod+pid / pod+conn /
// svc+node) of a fixed grid that dequeues items from a device-built work list (see
// k_probe_work). Keys of the pod and service tiers are few and skewed: most of the
// partitions are empty and a handful carry thousands of signals. Empty partitions get no
// item; a big signal list is sliced into items of kSigPerItem signals.
//
// Range accounting (why the pod tiers do not enumerate pairs). A signal's candidate spans
// in a tier are one contiguous range of the partition's (hash, ts)-sorted spans. When the
// hash run is uniform (same pod / pid / conn / svc|node / group) -- always, unless two keys
// collide -- the tier's contribution is arithmetic on that range:
//   pod+pid  (P2): all spans within 100 ms;
//   pod+conn (P3): spans within 250 ms minus the 100 ms sub-range when the pid matches
//                  (those pairs are P2's);
// counts go into a difference array (two LDS atomics per signal), incident sums add
// value x range length, the tier-4 overlap adds the range length. Pairs whose trace also
// matches (T1) are counted by their pod tier; the trace pass, which enumerates T1 exactly,
// skips counting those pairs and only contributes their (better) top-3 keys. Top-3 keys of
// pod-tier pairs are only needed for spans whose third-best is not yet a trace key
// ("needy" spans, usually none after the trace pass): those are visited through a compact
// needy list. Non-uniform runs fall back to the exact per-pair walk.
struct alignas(16) SpanKT {
  uint64_t h;
  int64_t t;
};
struct alignas(16) SpanTC {
  uint64_t tr;
  uint64_t cn;
};
struct alignas(16) SpanPP {
  uint32_t pod, pid, sn, grp;
};

constexpr int kLdsGroups = 64;
// Probe workgroups per phase (2 per CU) and signals per work item (a partition's list is sliced:
// staging repeats per item vs load balance). Round 6 sweep on the USER16 tree, K = 100, one box
// (profiles/r6_probe_sweep/): 512 x 6144 2.074 / 2.044 / 2.044 G events/s (chain 0.425-0.427 ms),
// 768 x 4096 (round 5's choice) 2.042 / 2.035 / 2.019 / 2.019 / 2.008 G (0.437-0.441 ms); 512 x
// 4096 2.02-2.05, 512 x 8192 2.004, 640 x 4096 2.010, 384 x 4096 1.959, x 2048 1.89-1.97.
constexpr int kProbeGrid = 512;
constexpr int kSigPerItem = 6144;

// Work list for the two probe phases, rebuilt every window on the device (no host sync,
// graph-capturable). One workgroup of kParts threads, one partition per thread:
//   work[0] / work[1]: item counts of phase 1 (trace) / phase 2 (pod+pid, pod+conn, svc+node)
//   work[2] / work[3]: dequeue counters (zeroed here)
//   items: code = key type << 30 | generation age << 28 | sole << 26 | partition << 16 | slice << 8 |
//          n slices (sole: the partition's only trace-phase item).
// Empty partitions get no item, so probe workgroups never wake for them; nor does a generation
// whose visible rows (ts >= its age's halo cut-off) all lie farther than the tier's window from
// every span of the window (typically the oldest generation at the pod tiers). Phase-2 items are
// placed longest first (LPT): a counting sort on an estimated cost class. The phase is a few
// thousand items of very different sizes (a staging cost per item, then up to kSigPerItem
// signals at a per-key-type rate) dequeued by kProbeGrid workgroups, so its makespan is set by the
// big items that start last; in key-type order the pod+conn items (the most expensive per
// signal) came after every pod+pid item and the phase ran ~2x its average load (probe
// profile). Results do not depend on item order: top-3 insertion is an atomic-min cascade
// and every count / sum is an integer atomic.
__device__ __forceinline__ uint32_t probe_item_class(int k, uint32_t n_sig, uint32_t n_span) {
  // cycles, fitted to the MISLO_PROBE_PROFILE counters (stage ~30 k, per-signal 40-90)
  constexpr uint32_t kPerSig[kKeyTypes] = {90, 40, 85, 60};
  const uint32_t cost = 24000u + 64u * min(n_span, 256u) + n_sig * kPerSig[k];
  return min(cost >> 13, 63u);
}

// (body: one workgroup of kParts threads; s / s2 = kParts words each, s_cls = 64 words of LDS)
__device__ __forceinline__ void probe_work_body(const uint32_t* __restrict__ span_base, const SignalCols& gc,
                                                const JoinParams& jp, int sig_per_item, uint32_t* __restrict__ work,
                                                unsigned long long* s, unsigned long long* s2, uint32_t* s_cls) {
  const int p = threadIdx.x;
  if (p < 64) s_cls[p] = 0u;
  const uint32_t cur = cur_slot(gc);
  const GenMeta* gm = gc.gen;
  // the window's span time range (without generations: no pruning)
  const int64_t s_lo = gm ? ts_of_image(gm->span_lo) : INT64_MIN, s_hi = gm ? ts_of_image(gm->span_hi) : INT64_MAX;
  uint32_t ns[kKeyTypes], ng[kKeyTypes][kMaxGens], n[kKeyTypes][kMaxGens], nk[kKeyTypes];
  // every list offset this thread may need, loaded up front: independent loads in flight together
  // instead of one dependent round trip per (key type, generation) behind the pruning tests
  uint32_t b_lo[kKeyTypes][kMaxGens], b_hi[kKeyTypes][kMaxGens];
#pragma unroll
  for (int a = 0; a < kMaxGens; ++a) {
    const uint32_t* b = gc.base + (size_t)(a < gc.gens ? age_slot(gc, cur, a) : 0u) * kBaseLen;
#pragma unroll
    for (int k = 0; k < kKeyTypes; ++k) {
      b_lo[k][a] = a < gc.gens ? b[k * kParts + p] : 0u;
      b_hi[k][a] = a < gc.gens ? b[k * kParts + p + 1] : 0u;
    }
  }
#pragma unroll
  for (int k = 0; k < kKeyTypes; ++k) {
    const int c = k * kParts + p;
    ns[k] = span_base[c + 1] - span_base[c];
    nk[k] = 0;
    const int64_t w = jp.win_ns[k];
#pragma unroll
    for (int a = 0; a < kMaxGens; ++a) {
      ng[k][a] = 0;
      n[k][a] = 0;
      if (a >= gc.gens || ns[k] == 0) continue;
      const uint32_t slot = age_slot(gc, cur, a);
      if (gm) {
        if ((uint32_t)a >= gm->filled || gm->tlo[slot] > gm->thi[slot]) continue;
        const int64_t lo = max(ts_of_image(gm->tlo[slot]), gm->cut[a]), hi = ts_of_image(gm->thi[slot]);
        if (lo > hi || hi < s_lo - w || lo > s_hi + w) continue;  // nothing visible can pair
      }
      ng[k][a] = b_hi[k][a] - b_lo[k][a];
      n[k][a] = ng[k][a] == 0 ? 0u : min((ng[k][a] + sig_per_item - 1) / (uint32_t)sig_per_item, (uint32_t)kProbeMaxSplit);
      nk[k] += n[k][a];
    }
  }
  // packed inclusive scans: trace | pod+pid and pod+conn | svc+node item counts, 32 bits each
  const unsigned long long mine = (unsigned long long)nk[0] | ((unsigned long long)nk[1] << 32);
  const unsigned long long mine2 = (unsigned long long)nk[2] | ((unsigned long long)nk[3] << 32);
  s[p] = mine;
  s2[p] = mine2;
  __syncthreads();
  for (int off = 1; off < kParts; off <<= 1) {
    const unsigned long long x = p >= off ? s[p - off] : 0ull, x2 = p >= off ? s2[p - off] : 0ull;
    __syncthreads();
    s[p] += x;
    s2[p] += x2;
    __syncthreads();
  }
  const unsigned long long tot = s[kParts - 1], tot2 = s2[kParts - 1], excl = s[p] - mine;
  const uint32_t t[kKeyTypes] = {(uint32_t)tot, (uint32_t)(tot >> 32), (uint32_t)tot2, (uint32_t)(tot2 >> 32)};
  uint32_t* items1 = work + 4;
  uint32_t* items2 = work + 4 + kProbePhaseItems;
  auto code = [&](int k, int a, uint32_t j) {
    return ((uint32_t)k << 30) | ((uint32_t)a << 28) | ((uint32_t)p << 16) | (j << 8) | n[k][a];
  };
  {
    uint32_t pos = (uint32_t)excl;
    const uint32_t sole = nk[0] == 1 ? 1u << 26 : 0u;
#pragma unroll
    for (int a = 0; a < kMaxGens; ++a)
      for (uint32_t j = 0; j < n[0][a]; ++j) items1[pos++] = code(0, a, j) | sole;
  }
  // phase 2: count items per cost class (slot 0 = most expensive), scan, place
  auto slice = [&](int k, int a, uint32_t j) {  // signals of slice j (k_probe's split rule)
    const uint32_t per = (ng[k][a] + n[k][a] - 1) / n[k][a];
    const uint32_t lo = j * per;
    return lo >= ng[k][a] ? 0u : min(ng[k][a], lo + per) - lo;
  };
#pragma unroll
  for (int k = 1; k < kKeyTypes; ++k)
#pragma unroll
    for (int a = 0; a < kMaxGens; ++a)
      for (uint32_t j = 0; j < n[k][a]; ++j) atomicAdd(&s_cls[63u - probe_item_class(k, slice(k, a, j), ns[k])], 1u);
  __syncthreads();
  if (p == 0) {
    uint32_t run = 0;
    for (int q = 0; q < 64; ++q) {
      const uint32_t v = s_cls[q];
      s_cls[q] = run;
      run += v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 1; k < kKeyTypes; ++k)
#pragma unroll
    for (int a = 0; a < kMaxGens; ++a)
      for (uint32_t j = 0; j < n[k][a]; ++j) {
        const uint32_t pos = atomicAdd(&s_cls[63u - probe_item_class(k, slice(k, a, j), ns[k])], 1u);
        items2[pos] = code(k, a, j);
      }
  if (p == 0) {
    work[0] = t[0];
    work[1] = t[1] + t[2] + t[3];
    work[2] = 0u;
    work[3] = 0u;
  }
}

__global__ __launch_bounds__(kParts) void k_probe_work(const uint32_t* __restrict__ span_base, SignalCols gc,
                                                       JoinParams jp, int sig_per_item, uint32_t* __restrict__ work) {
  __shared__ unsigned long long s[kParts], s2[kParts];
  __shared__ uint32_t s_cls[64];
  probe_work_body(span_base, gc, jp, sig_per_item, work, s, s2, s_cls);
}

// The signal scatter with the probe's work list built by one more workgroup of the same launch
// (block 0, dispatched first): the list needs only the span and signal list offsets, so it no
// longer runs alone between the scatter and the probe (~26 us of one CU, serial, per window).
// LDS is one buffer, used as either kernel's arrays.
template <int NT>
__global__ __launch_bounds__(NT) void k_scatter_sig_work(SignalCols gc, const int* __restrict__ n_ptr, int cap,
                                                         const uint32_t* __restrict__ part_off, int nblk_a,
                                                         const uint32_t* __restrict__ span_base, JoinParams jp,
                                                         int sig_per_item, uint32_t* __restrict__ work) {
  static_assert(NT == kParts, "the work-list block runs one thread per partition");
  static_assert(2 * kParts * 8 + 64 * 4 >= kKeyTypes * kParts * 4, "one LDS buffer serves both");
  __shared__ unsigned long long s_buf[2 * kParts + 32];
  if (blockIdx.x == 0) {
    probe_work_body(span_base, gc, jp, sig_per_item, work, s_buf, s_buf + kParts,
                    reinterpret_cast<uint32_t*>(s_buf + 2 * kParts));
    return;
  }
  scatter_sig_body<NT>(gc, n_ptr, cap, part_off, nblk_a, (int)blockIdx.x - 1, (int)gridDim.x - 1,
                       reinterpret_cast<uint32_t*>(s_buf));
}

// In-place inclusive scan of v[0..n), n <= 2 * NT (each thread owns two adjacent entries).
template <int NT>
__device__ __forceinline__ void block_inclusive_scan(int* v, int n, int* wsum) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int i0 = 2 * t, i1 = 2 * t + 1;
  const int a = i0 < n ? v[i0] : 0, b = i1 < n ? v[i1] : 0;
  const int local = a + b;
  int incl = local;
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(incl, off);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wave; ++w) base += wsum[w];
  const int excl = base + incl - local;
  if (i0 < n) v[i0] = excl + a;
  if (i1 < n) v[i1] = excl + a + b;
  __syncthreads();
}

// first index in [lo, hi) whose (h, t) is not less than (h0, t0)
__device__ __forceinline__ int lower_ht(const SpanKT* kt, int lo, int hi, uint64_t h0, int64_t t0) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const SpanKT e = kt[mid];
    if (less_ht(e.h, e.t, h0, t0)) lo = mid + 1; else hi = mid;
  }
  return lo;
}
// first index in [lo, hi) whose (h, t) is greater than (h0, t0)
__device__ __forceinline__ int upper_ht(const SpanKT* kt, int lo, int hi, uint64_t h0, int64_t t0) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const SpanKT e = kt[mid];
    if (less_ht(h0, t0, e.h, e.t)) hi = mid; else lo = mid + 1;
  }
  return lo;
}
__device__ __forceinline__ int lower_u16(const uint16_t* v, int n, int x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int)v[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Span staging, once per window: every (key type, partition) list of spans, in chunks of kChunk
// list positions, sorted by (key hash, ts) with its hash runs marked. The probe stages a list once
// per work item -- per generation and signal slice, 3-9 times a window -- and did this sort, the
// span gathers and the run scans each time; now it loads the chunk's PreSpans (coalesced).
// One workgroup per list: the kernel's time is its longest list's (the few service keys hold
// thousands of spans), so a workgroup owning several lists -- with a wave-level sort for the
// short ones -- ran slower (30.7 against 17.2 us, profiles/r3_kernels/step4_tried.md).
__device__ __forceinline__ void store_prespan(PreSpan* dst_p, uint64_t h, int64_t t, const SpanRec& rr, uint32_t idx,
                                              uint32_t run) {
  PreSpan ps;
  ps.h = h;
  ps.t = t;
  ps.tr = rr.tr;
  ps.cn = rr.cn;
  ps.pod = rr.pod;
  ps.pid = rr.pid;
  ps.sn = rr.sn;
  ps.grp = rr.grp;
  ps.idx = idx;
  ps.run = run;
  ps.pad[0] = ps.pad[1] = 0u;
  const uint4* src = reinterpret_cast<const uint4*>(&ps);
  uint4* dst = reinterpret_cast<uint4*>(dst_p);
#pragma unroll
  for (int q = 0; q < 4; ++q) dst[q] = src[q];
}

template <int NT>
__global__ __launch_bounds__(NT) void k_span_sort(SpanCols sc, const uint32_t* __restrict__ span_items,
                                                  const uint32_t* __restrict__ span_base, PreSpan* __restrict__ out) {
  static_assert(kChunk == NT, "one span per thread");
  __shared__ SpanKT s_kt[kChunk];
  __shared__ SpanTC s_tc[kChunk];
  __shared__ SpanPP s_pp[kChunk];
  __shared__ uint16_t s_pos[kChunk];
  __shared__ uint16_t s_inv[kChunk];
  __shared__ int s_aux[kChunk];
  __shared__ uint32_t s_ok[kChunk];
  __shared__ int s_wsum[NT / 64];
  const int c = blockIdx.x, k = c / kParts;
  const uint32_t sp0 = span_base[c], sp1 = span_base[c + 1];
  const int ti = threadIdx.x;
  for (uint32_t c0 = sp0; c0 < sp1; c0 += kChunk) {
    const int m = (int)min((uint32_t)kChunk, sp1 - c0);
    int M = 1;
    while (M < m) M <<= 1;
    __syncthreads();
    SpanRec rr{};
    uint32_t my_s = 0xFFFFFFFFu;
    if (ti < m) {
      my_s = span_items[c0 + ti];
      rr = sc.rec[my_s];
    }
    if (ti < M) {
      s_kt[ti] = ti < m ? SpanKT{key_hash(k, rr.tr, rr.pod, rr.pid, rr.cn, rr.sn), rr.ts} : SpanKT{~0ull, INT64_MAX};
      s_pos[ti] = (uint16_t)ti;  // pre-sort position, carried through the sort
    }
    __syncthreads();
    // bitonic sort of (hash, ts, position) ascending
    for (int size = 2; size <= M; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int t = threadIdx.x; t < (M >> 1); t += NT) {
          const int i = 2 * t - (t & (stride - 1));
          const int j = i + stride;
          const bool up = (i & size) == 0;
          const SpanKT ei = s_kt[i], ej = s_kt[j];
          const bool gt = less_ht(ej.h, ej.t, ei.h, ei.t);
          if (gt == up) {
            s_kt[i] = ej; s_kt[j] = ei;
            const uint16_t tp = s_pos[i]; s_pos[i] = s_pos[j]; s_pos[j] = tp;
          }
        }
        __syncthreads();
      }
    }
    if (ti < m) s_inv[s_pos[ti]] = (uint16_t)ti;
    __syncthreads();
    int i = 0;  // this thread's span, sorted position
    if (ti < m) {
      i = s_inv[ti];
      s_tc[i] = SpanTC{rr.tr, rr.cn};
      s_pp[i] = SpanPP{rr.pod, rr.pid, rr.sn, rr.grp};
      s_ok[i] = 1u;
      s_aux[i] = (i == 0 || s_kt[i].h != s_kt[i - 1].h) ? 1 : 0;  // hash-run heads
    }
    __syncthreads();
    block_inclusive_scan<NT>(s_aux, m, s_wsum);  // run id = #heads up to i, minus one
    if (ti < m && i > 0 && s_kt[i].h == s_kt[i - 1].h) {  // a run is uniform when its key fields agree
      const SpanPP a = s_pp[i], b = s_pp[i - 1];
      const SpanTC x = s_tc[i], y = s_tc[i - 1];
      if (a.pod != b.pod || a.pid != b.pid || a.sn != b.sn || a.grp != b.grp || (k == 2 && x.cn != y.cn))
        atomicAnd(&s_ok[s_aux[i] - 1], 0u);
    }
    __syncthreads();
    if (ti < m) {
      const uint32_t rid = (uint32_t)(s_aux[i] - 1);
      store_prespan(out + c0 + i, s_kt[i].h, s_kt[i].t, rr, my_s, rid | (s_ok[rid] << 16));
    }
  }
}

// LG: incident sums privatised in LDS (12 KB of the workgroup's 38 KB: 4 workgroups per CU);
// without, they go straight to the striped global copies and the probe fits 6 workgroups per CU.
template <int NT, bool LG>
__global__ __launch_bounds__(NT, LG ? 4 : 6) void k_probe(const PreSpan* __restrict__ pre,
                                              const uint32_t* __restrict__ span_base, SignalCols gc, int span_cap,
                                              JoinParams jp, unsigned long long* __restrict__ top3,
                                              uint32_t* __restrict__ cnt, int n_groups,
                                              unsigned long long* __restrict__ gsum, uint32_t* __restrict__ gcnt,
                                              unsigned long long* __restrict__ dbg, uint32_t* __restrict__ work,
                                              int phase) {
  // span fields packed 16 B per entry (one ds_read_b128 each)
  static_assert(kChunk == NT, "staging keeps one span per thread");
  __shared__ SpanKT s_kt[kChunk];
  __shared__ SpanTC s_tc[kChunk];
  __shared__ SpanPP s_pp[kChunk];
  __shared__ uint32_t s_i[kChunk];
  __shared__ unsigned long long s_top[kChunk * 3];
  __shared__ unsigned long long s_seed3[kChunk];  // global 3rd-best key after the trace pass
  __shared__ int s_diff[kChunk + 1];              // candidate counts (difference array)
  __shared__ int s_aux[kChunk];                   // scans: run ids, then needy positions
  __shared__ uint16_t s_rid[kChunk];              // hash-run id per sorted position
  __shared__ uint32_t s_runok[kChunk];            // hash run is uniform
  __shared__ uint16_t s_needy[kChunk];            // sorted positions of needy spans
  __shared__ int s_wsum[NT / 64];
  __shared__ int s_nneedy;
  __shared__ uint32_t s_item;
  constexpr int kLg = LG ? kLdsGroups * kSlots : 1;
  __shared__ unsigned long long s_gsum[kLg];
  __shared__ uint32_t s_gcnt[kLg];

  // incident sums go to one of kGroupStripes copies (folded after the join): thousands of
  // workgroups adding into the same G x 16 words would otherwise serialise in L2 atomics
  {
    const size_t stripe = (size_t)(blockIdx.x & (kGroupStripes - 1)) * (size_t)n_groups * kSlots;
    gsum += stripe;
    gcnt += stripe;
  }
  const bool grp_lds = LG && n_groups <= kLdsGroups;
  const bool any_groups = jp.group_mode == 1 && n_groups > 0;
  if (grp_lds && any_groups) {
    for (int i = threadIdx.x; i < kLdsGroups * kSlots; i += NT) {
      s_gsum[i] = 0ull;
      s_gcnt[i] = 0u;
    }
  }
  const bool cand1 = jp.conf[1] >= jp.threshold, cand2 = jp.conf[2] >= jp.threshold;
  unsigned long long n_cand = 0, n_low = 0, n_overlap = 0;
  const uint32_t n_work = work[phase];
  const uint32_t* items = work + 4 + (phase ? kProbePhaseItems : 0);
  const uint32_t cur = cur_slot(gc);

  // dynamic work queue: one item = (key type, partition, signal slice)
  for (;;) {
    __syncthreads();  // previous item's LDS reads are done before s_item / staging reuse
    if (threadIdx.x == 0) s_item = atomicAdd(&work[2 + phase], 1u);
    __syncthreads();
    const uint32_t it = s_item;
    if (it >= n_work) break;
#ifdef MISLO_PROBE_PROFILE
    unsigned long long pt = clock64(), p_stage = 0, p_sig = 0, p_flush = 0;
#endif
    const uint32_t code = items[it];
    const int k = (int)(code >> 30);
    const int age = (int)((code >> 28) & 3u);
    const int part = (int)((code >> 16) & 0x3FF);
    const uint32_t si = (code >> 8) & 0xFF, nsplit = code & 0xFF;
    const int c = k * kParts + part;
    const uint32_t sp0 = span_base[c], sp1 = span_base[c + 1];
    // the item's generation: its rows, lists and keys, its halo cut-off, and the row classes of
    // the top-3 key (this window's local rows, then older windows' local rows, then the other
    // GPUs' rows oldest first: the order of [rows | halo | remote] under nested halo selections)
    const uint32_t gslot = age_slot(gc, cur, age);
    const uint32_t* sig_base = gc.base + (size_t)gslot * kBaseLen;
    const uint32_t* sig_items = gc.items + (size_t)gslot * kKeyTypes * (size_t)gc.stride;
    const KeyTs* sig_keys = gc.keys + (size_t)gslot * kKeyTypes * (size_t)gc.stride;
    const SigRec* grec = gc.rec + (size_t)gslot * (size_t)gc.stride;
    const int64_t cut = gc.gen ? gc.gen->cut[age] : INT64_MIN;
    const uint32_t n_loc = gc.gen ? gc.gen->n_local[gslot] : 0xFFFFFFFFu;
    const uint32_t cls_loc = (uint32_t)age * (uint32_t)gc.stride;
    const uint32_t cls_rem = (uint32_t)(2 * gc.gens - 1 - age) * (uint32_t)gc.stride;
    const uint32_t gb0 = sig_base[c], gb1 = sig_base[c + 1];
    const uint32_t per = (gb1 - gb0 + nsplit - 1) / nsplit;
    const uint32_t sg0 = gb0 + si * per;
    const uint32_t sg1 = min(gb1, sg0 + per);

    const int64_t w = jp.win_ns[k];
    const bool cand_tier = jp.conf[k] >= jp.threshold;
    const bool count_only = (k == 3) && !cand_tier;          // broad tier: count, never enumerate
    const bool track_overlap = (k < 3) && (jp.conf[3] < jp.threshold);
    const bool do_groups = cand_tier && any_groups;
    const bool ranged = (k == 1 || k == 2);                  // range accounting tiers

    auto add_group = [&](uint32_t grp, int slot, unsigned long long milli, uint32_t n) {
      if (grp >= (uint32_t)n_groups || n == 0) return;
      if (grp_lds) {
        atomicAdd(&s_gsum[grp * kSlots + slot], milli * n);
        atomicAdd(&s_gcnt[grp * kSlots + slot], n);
      } else {
        atomicAdd(gsum + (size_t)grp * kSlots + slot, milli * n);
        atomicAdd(gcnt + (size_t)grp * kSlots + slot, n);
      }
    };
    auto add_range = [&](int a, int b) {  // +1 candidate for every span of [a, b)
      if (a < b) {
        atomicAdd(&s_diff[a], 1);
        atomicAdd(&s_diff[b], -1);
      }
    };

  for (uint32_t c0 = sp0; c0 < sp1; c0 += kChunk) {
    const int m = (int)min((uint32_t)kChunk, sp1 - c0);
    __syncthreads();
    // the chunk, sorted by k_span_sort: one span per thread at its sorted position
    const int ti = threadIdx.x;
    if (ti < m) {
      const uint4* src = reinterpret_cast<const uint4*>(pre + c0 + ti);
      const uint4 a = src[0], b = src[1], cc = src[2], d = src[3];
      const uint32_t my_s = d.x;
      s_kt[ti] = SpanKT{((uint64_t)a.y << 32) | a.x, (int64_t)(((uint64_t)a.w << 32) | a.z)};
      s_i[ti] = my_s;
      if (!count_only) {
        s_tc[ti] = SpanTC{((uint64_t)b.y << 32) | b.x, ((uint64_t)b.w << 32) | b.z};
        s_pp[ti] = SpanPP{cc.x, cc.y, cc.z, cc.w};
        s_top[3 * ti] = kEmpty;
        s_top[3 * ti + 1] = kEmpty;
        s_top[3 * ti + 2] = kEmpty;
        s_seed3[ti] = k > 0 ? top3[3ull * my_s + 2] : kEmpty;
        s_diff[ti] = 0;
        s_rid[ti] = (uint16_t)(d.y & 0xFFFFu);
        s_runok[d.y & 0xFFFFu] = d.y >> 16;  // every member of a run writes the same flag
      }
    }
    if (threadIdx.x == 0 && !count_only) s_diff[m] = 0;
    __syncthreads();  // the staged chunk is complete
    if (!count_only) {
      if (ranged) {
        // compact list of needy spans (sorted positions)
        for (int i = threadIdx.x; i < m; i += NT) {
          const unsigned long long seed = s_seed3[i];
          s_aux[i] = (cand_tier && (seed == kEmpty || (int)(seed >> 62) >= k)) ? 1 : 0;
        }
        __syncthreads();
        block_inclusive_scan<NT>(s_aux, m, s_wsum);
        for (int i = threadIdx.x; i < m; i += NT) {
          const int prev = i ? s_aux[i - 1] : 0;
          if (s_aux[i] != prev) s_needy[prev] = (uint16_t)i;
        }
        if (threadIdx.x == 0) s_nneedy = s_aux[m - 1];
        __syncthreads();
      }
    }
    const int n_needy = ranged && !count_only ? s_nneedy : 0;
#ifdef MISLO_PROBE_PROFILE
    { const unsigned long long t = clock64(); p_stage += t - pt; pt = t; }
#endif

    // The item's list entries -- (key hash, ts) and the row index, 20 coalesced bytes per lane --
    // stream kDepth iterations ahead. A signal's 48-byte row record (a random gather) is needed
    // only when its key run holds a span within the tier's window: the broad tier counts from
    // the keys alone, older generations' rows outside the halo and rows with no span in reach
    // cost no gather. A matching signal's search and gather are issued one iteration ahead of
    // its accounting, so the gather overlaps the previous signal's LDS work.
    constexpr int kDepth = 1;
    uint32_t q = sg0 + threadIdx.x;
    KeyTs kq[kDepth];
    uint32_t iq[kDepth];
#pragma unroll
    for (int d = 0; d < kDepth; ++d) {
      const bool ok = q + (d + 1) * NT < sg1;
      kq[d] = ok ? sig_keys[q + (d + 1) * NT] : KeyTs{0ull, INT64_MIN};
      iq[d] = ok ? sig_items[q + (d + 1) * NT] : 0u;
    }
    // stage 1 of an element: halo visibility, the span-run search, the record gather on a hit
    auto stage1 = [&](const KeyTs& e, uint32_t idx, bool valid, int& lo, bool& vis, bool& hit, SigHot& r) {
      vis = valid && e.t >= cut;
      hit = false;
      lo = 0;
      if (!vis) return;
      lo = lower_ht(s_kt, 0, m, e.h, e.t - w);
      if (count_only) return;
      hit = lo < m && s_kt[lo].h == e.h && s_kt[lo].t <= e.t + w;
      if (hit) r = load_hot(grec + idx);
    };
    KeyTs e0 = q < sg1 ? sig_keys[q] : KeyTs{0ull, INT64_MIN};
    uint32_t i0 = q < sg1 ? sig_items[q] : 0u;
    int lo0;
    bool vis0, hit0;
    SigHot r0{};
    stage1(e0, i0, q < sg1, lo0, vis0, hit0, r0);
    for (; q < sg1; q += NT) {
      const KeyTs e1 = kq[0];
      const uint32_t i1 = iq[0];
#pragma unroll
      for (int d = 0; d + 1 < kDepth; ++d) {
        kq[d] = kq[d + 1];
        iq[d] = iq[d + 1];
      }
      {
        const bool ok = q + (kDepth + 1) * NT < sg1;
        kq[kDepth - 1] = ok ? sig_keys[q + (kDepth + 1) * NT] : KeyTs{0ull, INT64_MIN};
        iq[kDepth - 1] = ok ? sig_items[q + (kDepth + 1) * NT] : 0u;
      }
      int lo1;
      bool vis1, hit1;
      SigHot r1{};
      stage1(e1, i1, q + NT < sg1, lo1, vis1, hit1, r1);
      // stage 2: this element's accounting
      do {
      if (!vis0) break;
      const uint64_t h = e0.h;
      const int64_t t = e0.t;
      const int lo = lo0;
      const int64_t thi = t + w;
      if (count_only) {
        n_low += (unsigned long long)(upper_ht(s_kt, lo, m, h, thi) - lo);
        break;
      }
      if (!hit0) break;
      const SigHot r = r0;
      const uint32_t g = (i0 < n_loc ? cls_loc : cls_rem) + i0;  // top-3 key row id
      const uint32_t g_pod = r.pod, g_pid = r.pid, g_sn = r.sn;
      const uint64_t g_tr = r.tr, g_cn = r.cn;
      const int g_slot = (int)r.slot;
      const unsigned long long g_milli = milli_units(r.val);
      const bool g_sn_ok = (g_sn >> 16) != 0 && (g_sn & 0xFFFF) != 0;

      // ---- range accounting (pod tiers, uniform hash run) ----------------------------
      if (ranged) {
        const SpanPP p0 = s_pp[lo];
        const SpanTC c0r = s_tc[lo];
        const bool key_ok = s_runok[s_rid[lo]] && p0.pod != 0 && p0.pod == g_pod &&
                            (k == 1 ? (p0.pid != 0 && p0.pid == g_pid) : (c0r.cn != 0 && c0r.cn == g_cn));
        if (key_ok) {
          const int hi = upper_ht(s_kt, lo, m, h, thi);
          int a1 = hi, b1 = hi;  // P2 sub-range excluded from the pod+conn tier
          if (k == 2 && p0.pid != 0 && p0.pid == g_pid) {
            a1 = lower_ht(s_kt, lo, hi, h, t - jp.win_ns[1]);
            b1 = upper_ht(s_kt, a1, hi, h, t + jp.win_ns[1]);
          }
          const int n_acc = (hi - lo) - (b1 - a1);
          if (n_acc > 0) {
            if (cand_tier) {
              add_range(lo, a1);
              add_range(b1, hi);
              n_cand += (unsigned long long)n_acc;
              if (do_groups) add_group(p0.grp, g_slot, g_milli, (uint32_t)n_acc);
            } else {
              n_low += (unsigned long long)n_acc;
            }
            if (track_overlap && g_sn_ok && p0.sn == g_sn && w <= jp.win_ns[3]) n_overlap += (unsigned long long)n_acc;
            // top-3 keys only for needy spans in the accepted ranges
            if (n_needy) {
              for (int part = 0; part < 2; ++part) {
                const int ra = part ? b1 : lo, rb = part ? hi : a1;
                for (int j = lower_u16(s_needy, n_needy, ra); j < n_needy && (int)s_needy[j] < rb; ++j) {
                  const int i = s_needy[j];
                  const SpanTC tc = s_tc[i];
                  if (tc.tr != 0 && tc.tr == g_tr) continue;  // a trace pair: its key is the trace pass's
                  const int64_t dt = iabs64(t - s_kt[i].t);
                  unsigned long long key = ((unsigned long long)k << 62) | ((unsigned long long)dt << kSigBits) |
                                           (unsigned long long)g;
                  if (key < s_seed3[i] && key < s_top[3 * i + 2]) {
#pragma unroll
                    for (int jj = 0; jj < 3; ++jj) {
                      const unsigned long long old = atomicMin(&s_top[3 * i + jj], key);
                      if (old == kEmpty) break;
                      key = old > key ? old : key;
                    }
                  }
                }
              }
            }
          }
          break;
        }
      }

      // ---- exact per-pair walk (trace tier, colliding / mixed runs, low threshold) ---
      uint32_t run_grp = 0xFFFFFFFFu, run_n = 0;
      for (int i = lo; i < m; ++i) {
        const SpanKT e = s_kt[i];
        if (e.h != h || e.t > thi) break;
        const int64_t dt = iabs64(t - e.t);
        const SpanTC tc = s_tc[i];
        const SpanPP pp = s_pp[i];
        const uint32_t p_pod = pp.pod;
        const uint64_t p_cn = tc.cn;
        const uint64_t p_tr = tc.tr;
        // exact key equality (hash collision guard)
        if (k == 0 && p_tr != g_tr) continue;
        if (k == 1 && !(p_pod == g_pod && pp.pid == g_pid)) continue;
        if (k == 2 && !(p_pod == g_pod && p_cn == g_cn)) continue;
        const bool in_p2 = p_pod != 0 && p_pod == g_pod && pp.pid != 0 && pp.pid == g_pid && dt <= jp.win_ns[1];
        const bool in_p3 = p_pod != 0 && p_pod == g_pod && p_cn != 0 && p_cn == g_cn && dt <= jp.win_ns[2];
        const bool trace_eq = p_tr != 0 && p_tr == g_tr;
        // REF tier precedence: a pair belongs to the first tier it satisfies
        if (k == 2 && in_p2) continue;                        // P2's pair
        if (k == 3 && (trace_eq || in_p2 || in_p3)) continue;  // higher tiers' pairs
        // pod tiers count their trace pairs too (range accounting); the trace tier then
        // leaves the counting of those pairs to them and only contributes the key
        int owner = k;
        if (k == 0) owner = in_p2 ? 1 : (in_p3 ? 2 : 0);
        const bool tier_cand = jp.conf[k] >= jp.threshold;
        const bool insert_key = tier_cand && !(k >= 1 && trace_eq);
        if (insert_key) {
          unsigned long long key = ((unsigned long long)k << 62) | ((unsigned long long)dt << kSigBits) |
                                   (unsigned long long)g;
          if (key < s_seed3[i] && key < s_top[3 * i + 2]) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              const unsigned long long old = atomicMin(&s_top[3 * i + j], key);
              if (old == kEmpty) break;
              key = old > key ? old : key;
            }
          }
        }
        // counting: by the owning tier's accounting, fixed up when confidence classes differ
        bool count_cand = false, count_low = false, fix_low = false, count_ovl = false;
        if (owner == k) {
          count_cand = tier_cand;
          count_low = !tier_cand;
          count_ovl = track_overlap;
        } else {  // k == 0, pair already counted by pod tier `owner`
          const bool owner_cand = owner == 1 ? cand1 : cand2;
          if (tier_cand && !owner_cand) {
            count_cand = true;
            fix_low = true;
          }
        }
        if (count_cand) {
          atomicAdd(&s_diff[i], 1);
          atomicAdd(&s_diff[i + 1], -1);
          ++n_cand;
          if (fix_low) --n_low;
          if (do_groups || (k == 0 && any_groups)) {
            const uint32_t grp = pp.grp;
            if (grp != run_grp) {
              add_group(run_grp, g_slot, g_milli, run_n);
              run_grp = grp;
              run_n = 0;
            }
            ++run_n;
          }
        } else if (count_low) {
          ++n_low;
        }
        if (count_ovl) {
          const uint32_t p_sn = pp.sn;
          if ((p_sn >> 16) != 0 && (p_sn & 0xFFFF) != 0 && p_sn == g_sn && dt <= jp.win_ns[3]) ++n_overlap;
        }
      }
      add_group(run_grp, g_slot, g_milli, run_n);
      } while (0);
      e0 = e1;
      i0 = i1;
      lo0 = lo1;
      vis0 = vis1;
      hit0 = hit1;
      r0 = r1;
    }
    // flush this chunk's per-span candidates to the global top-3 / counts
    __syncthreads();
#ifdef MISLO_PROBE_PROFILE
    { const unsigned long long t = clock64(); p_sig += t - pt; pt = t; }
#endif
    if (!count_only) {
      block_inclusive_scan<NT>(s_diff, m, s_wsum);  // difference array -> per-span counts
      // phase 1, sole item of its partition (one slice of one generation): the only writer of
      // these spans so far (a span has one trace key), so plain stores replace the atomic cascade
      const bool sole = phase == 0 && ((code >> 26) & 1u);
      for (int i = threadIdx.x; i < m; i += NT) {
        const int nc = s_diff[i];
        const uint32_t s = s_i[i];
        if (sole) {
          cnt[s] = (uint32_t)nc;
#pragma unroll
          for (int j = 0; j < 3; ++j) top3[3ull * s + j] = s_top[3 * i + j];
          continue;
        }
        if (nc) atomicAdd(cnt + s, (uint32_t)nc);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const unsigned long long key = s_top[3 * i + j];
          if (key == kEmpty) break;
          top3_insert(top3 + 3ull * s, key);
        }
      }
    }
#ifdef MISLO_PROBE_PROFILE
    __syncthreads();
    { const unsigned long long t = clock64(); p_flush += t - pt; pt = t; }
#endif
  }
#ifdef MISLO_PROBE_PROFILE
  // per key type: items, signals, span chunks, stage / signal-loop / flush cycles
  if (threadIdx.x == 0) {
    unsigned long long* pr = reinterpret_cast<unsigned long long*>(work + kProbeProfOff) + 8 * k;
    atomicAdd(pr + 0, 1ull);
    atomicAdd(pr + 1, (unsigned long long)(sg1 - sg0));
    atomicAdd(pr + 2, (unsigned long long)((sp1 - sp0 + kChunk - 1) / kChunk));
    atomicAdd(pr + 3, p_stage);
    atomicAdd(pr + 4, p_sig);
    atomicAdd(pr + 5, p_flush);
  }
#endif
  }  // work loop
  if (grp_lds && any_groups) {
    __syncthreads();
    for (int i = threadIdx.x; i < n_groups * kSlots; i += NT) {
      const uint32_t n = s_gcnt[i];
      if (n) {
        atomicAdd(gsum + i, s_gsum[i]);
        atomicAdd(gcnt + i, n);
      }
    }
  }
  // wave reduce, one atomic per wave (n_low may go transiently negative per lane: two's
  // complement wrap is exact in the final unsigned sum)
  for (int off = 32; off > 0; off >>= 1) {
    n_cand += __shfl_xor(n_cand, off);
    n_low += __shfl_xor(n_low, off);
    n_overlap += __shfl_xor(n_overlap, off);
  }
  if ((threadIdx.x & 63) == 0) {
    if (n_cand) atomicAdd(&dbg[0], n_cand);
    if (n_low) atomicAdd(&dbg[1], n_low);
    if (n_overlap) atomicAdd(&dbg[2], n_overlap);
  }
}

// ---------------------------------------------------------------------------------------
// finalize: top-3 -> attribute max-merge, confidence, retrieval decomposition, groups
// ---------------------------------------------------------------------------------------

template <int NT>
__global__ __launch_bounds__(NT) void k_finalize(const int* __restrict__ ns_ptr, int span_cap,
                                                 const unsigned long long* __restrict__ top3,
                                                 const uint32_t* __restrict__ cnt, SignalCols gc, SpanCols sc,
                                                 JoinParams jp, const float* __restrict__ base_attrs,
                                                 float* __restrict__ attrs, float* __restrict__ conf,
                                                 float* __restrict__ kernel_ms, int n_groups,
                                                 unsigned long long* __restrict__ gsum, uint32_t* __restrict__ gcnt,
                                                 unsigned long long* __restrict__ dbg) {
  const int ns = min(*ns_ptr, span_cap);
  const int s = blockIdx.x * NT + threadIdx.x;
  {
    const size_t stripe = (size_t)(blockIdx.x & (kGroupStripes - 1)) * (size_t)n_groups * kSlots;
    gsum += stripe;
    gcnt += stripe;
  }
  unsigned long long dropped = 0, enriched = 0;
  const uint32_t cur = cur_slot(gc);
  if (s < ns) {
    float a[kSlots];
#pragma unroll
    for (int j = 0; j < kSlots; ++j) a[j] = base_attrs ? base_attrs[(size_t)s * kSlots + j] : __builtin_nanf("");
    float mc = 0.f;
    const int keep = jp.fanout;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const unsigned long long key = top3[3ull * s + j];
      if (key == kEmpty || j >= keep) continue;
      const int tier = (int)(key >> 62);
      // the key's row id: class * stride + row, class = generation age for local rows and
      // 2 * gens - 1 - age for the other GPUs' rows (k_probe)
      const uint32_t g = (uint32_t)(key & ((1ull << kSigBits) - 1));
      const uint32_t cls = g / (uint32_t)gc.stride, row = g - cls * (uint32_t)gc.stride;
      const int age = (int)cls < gc.gens ? (int)cls : 2 * gc.gens - 1 - (int)cls;
      const SigRec& r = gc.rec[(size_t)age_slot(gc, cur, age) * (size_t)gc.stride + row];
      const int slot = (int)r.slot;
      const float v = r.val;
      // REF merge: attr = value if absent or value > existing
      float cur = a[0];
#pragma unroll
      for (int q = 0; q < kSlots; ++q) if (q == slot) cur = a[q];
      const bool take = (cur != cur) || v > cur;
#pragma unroll
      for (int q = 0; q < kSlots; ++q) if (q == slot && take) a[q] = v;
      mc = fmaxf(mc, jp.conf[tier]);
    }
    const uint32_t c = cnt[s];
    if ((int)c > keep) dropped = c - keep;
    if (mc > 0.f) enriched = 1;
    conf[s] = mc;
    // retrieval decomposition (REF correlator.go:179-194): dns + connect + tls
    float km = 0.f;
    if (a[0] == a[0]) km += a[0];
    if (a[3] == a[3]) km += a[3];
    if (a[5] == a[5]) km += a[5];
    kernel_ms[s] = km > 0.f ? km : __builtin_nanf("");
#pragma unroll
    for (int j = 0; j < kSlots; ++j) attrs[(size_t)s * kSlots + j] = a[j];
    const uint32_t grp = sc.rec[s].grp;
    if (jp.group_mode == 0 && n_groups > 0 && grp < (uint32_t)n_groups) {
#pragma unroll
      for (int j = 0; j < kSlots; ++j) {
        if (a[j] == a[j]) {
          atomicAdd(gsum + (size_t)grp * kSlots + j, milli_units(a[j]));
          atomicAdd(gcnt + (size_t)grp * kSlots + j, 1u);
        }
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    dropped += __shfl_xor(dropped, off);
    enriched += __shfl_xor(enriched, off);
  }
  if ((threadIdx.x & 63) == 0) {
    if (dropped) atomicAdd(&dbg[3], dropped);
    if (enriched) atomicAdd(&dbg[4], enriched);
  }
}

__device__ __forceinline__ float group_feature(unsigned long long sum, uint32_t c) {
  // exact integer sums of milli-unit values: deterministic under any atomic order and
  // associative across ranks (the group-sum all-reduce); oracle.join computes the same
  return c ? (float)(((double)sum * 1e-3) / (double)c) : __builtin_nanf("");
}

// Sum the incident-sum stripes into stripe 0 (exact integers: order-free) and write the
// rank-local incident features in the same pass (global scope recomputes them from the
// all-reduced sums with k_group_features).
__global__ __launch_bounds__(256) void k_fold_groups(int n, unsigned long long* __restrict__ gsum,
                                                     uint32_t* __restrict__ gcnt, float* __restrict__ feat) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  unsigned long long s = gsum[i];
  uint32_t c = gcnt[i];
#pragma unroll
  for (int r = 1; r < kGroupStripes; ++r) {
    s += gsum[(size_t)r * n + i];
    c += gcnt[(size_t)r * n + i];
  }
  gsum[i] = s;
  gcnt[i] = c;
  feat[i] = group_feature(s, c);
}

__global__ __launch_bounds__(256) void k_group_features(int n, const unsigned long long* __restrict__ gsum,
                                                        const uint32_t* __restrict__ gcnt, float* __restrict__ feat) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  feat[i] = group_feature(gsum[i], gcnt[i]);
}

// ---------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------

static int probe_item_signals() {  // MISLO_PROBE_ITEM: signals per work item (diagnostic)
  static const int per_item = [] {
    const char* v = getenv("MISLO_PROBE_ITEM");
    const int x = v ? atoi(v) : kSigPerItem;
    return x >= 1 ? x : kSigPerItem;
  }();
  return per_item;
}

void launch_partition_sig(const SignalCols& gc, const int* n_dev, int cap, int nblk, const uint32_t* part_blk,
                          uint32_t* part_off, uint32_t* part_tot, hipStream_t stream, int nblk_a, hipEvent_t bases_done,
                          const uint32_t* work_span_base, const JoinParams* work_jp, uint32_t* work) {
  hipLaunchKernelGGL(k_part_scan, dim3(kKeyTypes * kParts / kScanCols), dim3(kScanCols * kScanRG), 0, stream,
                     part_blk, nblk, part_off, part_tot);
  hipLaunchKernelGGL(k_base_scan, dim3(1), dim3(kBaseNT), 0, stream, part_tot, gc.base, gc.gen);
  if (bases_done) (void)hipEventRecord(bases_done, stream);  // the span branch's probe work list may start
  const int na = nblk_a > 0 && nblk_a < nblk ? nblk_a : nblk;
  if (work != nullptr && work_jp != nullptr && work_span_base != nullptr)  // + the probe's work list
    hipLaunchKernelGGL((k_scatter_sig_work<1024>), dim3(nblk + 1), dim3(1024), 0, stream, gc, n_dev, cap, part_off,
                       na, work_span_base, *work_jp, probe_item_signals(), work);
  else
    hipLaunchKernelGGL((k_scatter_sig<1024>), dim3(nblk), dim3(1024), 0, stream, gc, n_dev, cap, part_off, na);
}

void launch_partition(const PartCodes* codes, const int* n_dev, int cap, int nblk, const uint32_t* part_blk,
                      uint32_t* part_off, uint32_t* part_tot, uint32_t* part_base, uint32_t* items,
                      hipStream_t stream, int nblk_a) {
  static_assert((kKeyTypes * kParts) % kScanCols == 0, "scan columns tile the partition matrix");
  hipLaunchKernelGGL(k_part_scan, dim3(kKeyTypes * kParts / kScanCols), dim3(kScanCols * kScanRG), 0, stream,
                     part_blk, nblk, part_off, part_tot);
  hipLaunchKernelGGL(k_base_scan, dim3(1), dim3(kBaseNT), 0, stream, part_tot, part_base, nullptr);
  // 1024 threads per workgroup: the grid is one workgroup per decode block (<= 256), so 256
  // threads left 4 waves per CU to hide the scattered stores and LDS atomics
  hipLaunchKernelGGL((k_scatter<1024>), dim3(nblk), dim3(1024), 0, stream, codes, n_dev, cap, part_off, part_base,
                     items, nblk_a > 0 && nblk_a < nblk ? nblk_a : nblk);
}

void launch_probe(const SpanCols& sc, const uint32_t* span_items, const uint32_t* span_base, const SignalCols& gc,
                  int span_cap, const JoinParams& jp, unsigned long long* top3, uint32_t* cnt, int n_groups,
                  unsigned long long* gsum, uint32_t* gcnt, unsigned long long* dbg, uint32_t* work,
                  PreSpan* span_pre, hipStream_t stream) {
  // phase 1: trace tier; phase 2: pod+pid, pod+conn, svc+node seeded with phase 1's top-3.
  // Both phases pull items from the device-built work list. Diagnostic knobs (read once):
  // MISLO_PROBE_GRID workgroups per phase, MISLO_PROBE_ITEM signals per work item.
  static const int grid = [] {
    const char* v = getenv("MISLO_PROBE_GRID");
    const int x = v ? atoi(v) : kProbeGrid;
    return x >= 1 && x <= 65536 ? x : kProbeGrid;
  }();
  static const int per_item = [] {
    const char* v = getenv("MISLO_PROBE_ITEM");
    const int x = v ? atoi(v) : kSigPerItem;
    return x >= 1 ? x : kSigPerItem;
  }();
  (void)sc, (void)span_items, (void)per_item;
  static const bool lds_groups = [] {  // MISLO_PROBE_LDS_GROUPS=0: sums to global memory, 6 WG/CU
    const char* v = getenv("MISLO_PROBE_LDS_GROUPS");
    return !(v && atoi(v) == 0);
  }();
  for (int phase = 0; phase < 2; ++phase) {
    if (lds_groups)
      hipLaunchKernelGGL((k_probe<256, true>), dim3(grid), dim3(256), 0, stream, span_pre, span_base, gc, span_cap, jp,
                         top3, cnt, n_groups, gsum, gcnt, dbg, work, phase);
    else
      hipLaunchKernelGGL((k_probe<256, false>), dim3(grid), dim3(256), 0, stream, span_pre, span_base, gc, span_cap, jp,
                         top3, cnt, n_groups, gsum, gcnt, dbg, work, phase);
  }
}

void launch_span_sort(const SpanCols& sc, const uint32_t* span_items, const uint32_t* span_base, PreSpan* span_pre,
                      hipStream_t stream) {
  hipLaunchKernelGGL((k_span_sort<kChunk>), dim3(kKeyTypes * kParts), dim3(kChunk), 0, stream, sc, span_items,
                     span_base, span_pre);
}

void launch_probe_work(const uint32_t* span_base, const SignalCols& gc, const JoinParams& jp, uint32_t* work,
                       hipStream_t stream) {
  hipLaunchKernelGGL(k_probe_work, dim3(1), dim3(kParts), 0, stream, span_base, gc, jp, probe_item_signals(), work);
}

void launch_finalize(const int* ns_dev, int span_cap, const unsigned long long* top3, const uint32_t* cnt,
                     const SignalCols& gc, const SpanCols& sc, const JoinParams& jp, const float* base_attrs,
                     float* attrs, float* conf, float* kernel_ms, int n_groups, unsigned long long* gsum, uint32_t* gcnt,
                     float* feat, unsigned long long* dbg, hipStream_t stream) {
  hipLaunchKernelGGL((k_finalize<256>), dim3((span_cap + 255) / 256), dim3(256), 0, stream, ns_dev, span_cap, top3,
                     cnt, gc, sc, jp, base_attrs, attrs, conf, kernel_ms, n_groups, gsum, gcnt, dbg);
  if (n_groups > 0) {
    const int n = n_groups * kSlots;
    hipLaunchKernelGGL(k_fold_groups, dim3((n + 255) / 256), dim3(256), 0, stream, n, gsum, gcnt, feat);
  }
}

// Incident features from (possibly all-reduced) per-group sums: the second half of a
// window in global incident scope (parallel/__init__.py).
void launch_group_features(int n_groups, const unsigned long long* gsum, const uint32_t* gcnt, float* feat, hipStream_t stream) {
  if (n_groups <= 0) return;
  const int n = n_groups * kSlots;
  hipLaunchKernelGGL(k_group_features, dim3((n + 255) / 256), dim3(256), 0, stream, n, gsum, gcnt, feat);
}

}  // namespace mislo
