// Window-to-window and GPU-to-GPU rows of the native engine.
//
//   halo   : window k+1 also joins the decoded rows of earlier windows whose timestamps lie within
//            halo_ms of the latest local record of every window since (REF correlates against a
//            continuous 2 s buffer, pkg/correlation/dns.go:12), so a span early in window k+1
//            still finds the signals recorded just before the cut. The rows stay where their own
//            window decoded them: the engine keeps up to kMaxGens generations of rows, partition
//            lists and list keys resident, and k_gen_begin turns the generations' anchors into
//            per-age visibility cut-offs that the probe applies while it streams the lists (the
//            rows a chain of per-window halo selections would carry forward, with no copy, no
//            re-decode and no re-partition of them).
//   remote : each GPU's trace-tagged local rows of window k at warn level or above (the
//            evidence; identity dropped: only their trace hash can join) are all-gathered over
//            RCCL as 24-byte XRecs and appended to the same window's rows on
//            every other GPU, so a request traced across nodes joins the elevated signals of
//            every node that saw it.
//
// The trace-row selection is a stable stream compaction (count -> exclusive scan -> ordered
// scatter), so the exchanged rows, and with them the join's tie-breaks by row, are deterministic.
// By default the count is fused into segment 0's decode (per-block counts and 64-row ballot
// masks) and the scatter reads only the selected rows (k_sel_scatter_mask); the two full passes
// (k_sel_count, k_sel_scatter) remain behind MISLO_SEL_TWO_PASS=1.
#include "mislo_common.h"
#include "mislo_launch.h"
#include "mislo_packet.h"

namespace mislo {

namespace {

constexpr int kSelNT = 256;

struct SelArgs {
  SignalCols gc;        // the current generation's rows
  const int* rows;      // rows[0] = local rows of the window
  const int* counts;    // counts[0] = local rows
  int cap;
};

__device__ __forceinline__ int sel_end(const SelArgs& a) { return min(a.counts[0], min(a.rows[0], a.cap)); }

__device__ __forceinline__ const SigRec* sel_rows(const SelArgs& a) {
  return a.gc.rec + (size_t)cur_slot(a.gc) * (size_t)a.gc.stride;
}

// a warn-level (or worse) trace-tagged joinable local row
__device__ __forceinline__ bool selected(const SelArgs& a, const SigRec& r, int i) {
  if (r.slot == kNoSlot || r.ts == 0) return false;
  return r.tr != 0 && a.gc.status[i] >= 1;
}

// per-block counts of selected rows (fixed grid; block b owns a contiguous chunk)
__global__ __launch_bounds__(kSelNT) void k_sel_count(SelArgs a, uint32_t* __restrict__ blk_cnt) {
  const int n = sel_end(a);
  const SigRec* rec = sel_rows(a);
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);
  uint32_t c = 0;
  for (int i = beg + threadIdx.x; i < end; i += kSelNT) c += selected(a, rec[i], i) ? 1u : 0u;
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  __shared__ uint32_t s_w[kSelNT / 64];
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kSelNT / 64; ++w) t += s_w[w];
    blk_cnt[blockIdx.x] = t;
  }
}

// exclusive scan of <= 1024 block counts; total (clamped to the output capacity) -> *n_out, the
// rows beyond the capacity -> *dropped (the packet's dbg[kDbgXchgDropped]: never silent)
__global__ __launch_bounds__(1024) void k_sel_scan(const uint32_t* __restrict__ blk_cnt, int nblk,
                                                  uint32_t* __restrict__ blk_off, uint32_t* __restrict__ n_out,
                                                  uint32_t out_cap, unsigned long long* __restrict__ dropped) {
  __shared__ uint32_t s[1024];
  const int t = threadIdx.x;
  const uint32_t v = t < nblk ? blk_cnt[t] : 0u;
  s[t] = v;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const uint32_t x = t >= off ? s[t - off] : 0u;
    __syncthreads();
    s[t] += x;
    __syncthreads();
  }
  if (t < nblk) blk_off[t] = s[t] - v;
  if (t == 1023) {
    *n_out = min(s[1023], out_cap);
    if (dropped && s[1023] > out_cap) atomicAdd(dropped, (unsigned long long)(s[1023] - out_cap));
  }
}

// ordered scatter: block offset + wave offsets + in-wave ballot rank; 24-byte exchange rows
// (XRec: no identity)
__global__ __launch_bounds__(kSelNT) void k_sel_scatter(SelArgs a, const uint32_t* __restrict__ blk_off,
                                                        XRec* __restrict__ out, uint32_t out_cap) {
  const int n = sel_end(a);
  const SigRec* rec = sel_rows(a);
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);
  __shared__ uint32_t s_w[kSelNT / 64];
  __shared__ uint32_t s_base;
  if (threadIdx.x == 0) s_base = blk_off[blockIdx.x];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int trips = end > beg ? (end - beg + kSelNT - 1) / kSelNT : 0;
  for (int it = 0; it < trips; ++it) {
    const int i = beg + it * kSelNT + threadIdx.x;
    SigRec r{};
    bool s = false;
    if (i < end) {
      r = rec[i];
      s = selected(a, r, i);
    }
    const unsigned long long m = __ballot(s);
    const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();  // s_base of the previous trip is final
    if (lane == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t wo = s_base;
    for (int q = 0; q < w; ++q) wo += s_w[q];
    if (s) {
      const uint32_t dst = wo + rank;
      if (dst < out_cap) out[dst] = XRec{r.ts, r.tr, r.val, r.slot};  // joins by its trace hash only
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int q = 0; q < kSelNT / 64; ++q) t += s_w[q];
      s_base += t;
    }
  }
}

// ordered scatter from segment 0's decode (fused selection): the decode's geometry (its grid,
// kDecodeNT threads, block b owning rows [b * chunk, ...) of [0, min(rows[0], cap))), its ballot
// mask per (block, trip, wave) and its per-block count (scanned into blk_off). Only the selected
// rows are read.
template <int NT>
__global__ __launch_bounds__(NT) void k_sel_scatter_mask(SignalCols gc, const int* __restrict__ rows, int cap,
                                                         const unsigned long long* __restrict__ mask, int mask_stride,
                                                         const uint32_t* __restrict__ blk_off, XRec* __restrict__ out,
                                                         uint32_t out_cap) {
  constexpr int NW = NT / 64;
  const int n = min(rows[0], cap);
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);
  const int trips = end > beg ? (end - beg + NT - 1) / NT : 0;
  const SigRec* rec = gc.rec + (size_t)cur_slot(gc) * (size_t)gc.stride;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ uint32_t s_w[NW];
  uint32_t base = blk_off[blockIdx.x];
  const unsigned long long* mb = mask + (size_t)blockIdx.x * mask_stride;
  for (int it = 0; it < trips; ++it) {
    const unsigned long long m = mb[it * NW + w];
    if (lane == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t wo = base, tot = 0;
    for (int q = 0; q < NW; ++q) {
      if (q < w) wo += s_w[q];
      tot += s_w[q];
    }
    if ((m >> lane) & 1ull) {
      const uint32_t dst = wo + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      const SigRec r = rec[beg + it * NT + threadIdx.x];
      if (dst < out_cap) out[dst] = XRec{r.ts, r.tr, r.val, r.slot};  // joins by its trace hash only
    }
    base += tot;
    __syncthreads();  // s_w is rewritten by the next trip
  }
}

// other GPUs' exchanged rows (each rank's block: a 24-byte header holding its row count, then
// XRec rows) as identity-free SigRecs, in rank order: appended to the window's own rows
// Rows that do not fit are counted, never silently lost: a block's rows beyond the all-gathered
// block size (its sender selected more than was sent) into dropped[0] (dbg[kDbgXchgDropped], by
// the sender's successor only, so the node-wide sum counts each row once), rows beyond the import
// capacity into dropped[1] (dbg[kDbgImportDropped]).
__global__ __launch_bounds__(256) void k_remote_merge(const uint8_t* __restrict__ xrecv, size_t stride, int world,
                                                      int me, SigRec* __restrict__ imp,
                                                      uint32_t* __restrict__ remote_n, uint32_t imp_cap,
                                                      unsigned long long* __restrict__ dropped) {
  uint32_t off = 0;
  const uint32_t per_blk = (uint32_t)((stride - sizeof(XRec)) / sizeof(XRec));
  for (int r = 0; r < world; ++r) {
    if (r == me) continue;
    const uint8_t* blk = xrecv + (size_t)r * stride;
    const uint32_t hdr = *reinterpret_cast<const uint32_t*>(blk);
    const uint32_t c = min(hdr, per_blk);
    if (dropped && hdr > c && (r + 1) % world == me && blockIdx.x == 0 && threadIdx.x == 0)
      atomicAdd(&dropped[0], (unsigned long long)(hdr - c));
    const XRec* rows = reinterpret_cast<const XRec*>(blk + sizeof(XRec));
    for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < c; j += gridDim.x * 256)
      if (off + j < imp_cap) {
        const XRec x = rows[j];
        SigRec r{};
        r.ts = x.ts;
        r.tr = x.tr;
        r.val = x.val;
        r.slot = x.slot;
        imp[off + j] = r;
      }
    off += c;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *remote_n = off < imp_cap ? off : imp_cap;
    if (dropped && off > imp_cap) atomicAdd(&dropped[1], (unsigned long long)(off - imp_cap));
  }
}

// rows of the window: rows[0] = local records (decode segment 0), rows[1] = rows[0] + other
// GPUs' rows (segment 1); the generation keeps both counts (the join's row classes)
__device__ __forceinline__ void window_rows_body(const int* __restrict__ counts, uint32_t remote_n, int cap,
                                                 int* __restrict__ rows, GenMeta* __restrict__ gen) {
  const long long r0 = counts[0] < cap ? counts[0] : cap;
  const long long b = r0 + remote_n;
  rows[0] = (int)r0;
  rows[1] = (int)(b < cap ? b : cap);
  if (gen) {
    gen->n_local[gen->cur] = (uint32_t)rows[0];
    gen->n_rows[gen->cur] = (uint32_t)rows[1];
  }
}

__global__ void k_window_rows(const int* __restrict__ counts, const uint32_t* __restrict__ remote_n, int cap,
                              int* __restrict__ rows, GenMeta* __restrict__ gen) {
  if (threadIdx.x == 0) window_rows_body(counts, *remote_n, cap, rows, gen);
}

// Start of a window: the finished window's halo anchor (its latest local record), the next
// slot (its old rows, kMaxGens windows back, drop out), and the visibility cut-off of every
// age: a row of window k - a stays visible in window k while ts >= tmax_i - halo for every
// window i in [k - a, k - 1] (a window without local records ends the chain, as an empty
// selection would).
__device__ __forceinline__ void gen_begin_body(GenMeta* __restrict__ g, unsigned long long tmax_prev, int gens,
                                               long long halo_ns) {
  if (g->filled > 0) g->tmax_local[g->cur] = (int64_t)tmax_prev;
  const uint32_t cur = (g->cur + 1) % (uint32_t)gens;
  g->cur = cur;
  g->filled = min(g->filled + 1, (uint32_t)gens);
  g->n_local[cur] = 0;
  g->n_rows[cur] = 0;
  g->tmax_local[cur] = 0;
  g->tlo[cur] = ~0ull;
  g->thi[cur] = 0ull;
  g->span_lo = ~0ull;
  g->span_hi = 0ull;
  g->cut[0] = INT64_MIN;
  bool ok = halo_ns > 0;
  int64_t c = INT64_MIN;
  for (int a = 1; a < kMaxGens; ++a) {
    if (ok && a < gens && (uint32_t)a < g->filled) {
      const int64_t tm = g->tmax_local[(cur + (uint32_t)(gens - a)) % (uint32_t)gens];
      if (tm == 0) ok = false;
      else c = max(c, tm - (int64_t)halo_ns);
    } else {
      ok = false;
    }
    g->cut[a] = ok ? c : INT64_MAX;
  }
}

// The head of a window's graph in ONE dispatch (it was four latency-bound ones: generation
// step, accumulator fill, ring-state fill, row counts -- ~19 us per window): every thread zeroes
// the accumulators while thread 0 of block 0 runs the ordered scalar part -- the finished
// window's tmax into its generation, then tmax reset; the ring state (first busy record: none);
// no other GPUs' rows yet; the window's row counts.
__global__ __launch_bounds__(256) void k_window_begin(FillList fl, GenMeta* __restrict__ gen,
                                                      unsigned long long* __restrict__ tmax, int gens, long long halo_ns,
                                                      uint32_t* __restrict__ ring_state, uint32_t* __restrict__ remote_n,
                                                      const int* __restrict__ counts, int cap, int* __restrict__ rows) {
  for (int q = 0; q < fl.count; ++q) {
    const FillSeg sg = fl.seg[q];
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < sg.n; i += gridDim.x * 256) sg.ptr[i] = sg.value;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (gen) gen_begin_body(gen, *tmax, gens, halo_ns);
    *tmax = 0ull;
    ring_state[kRsFirstBusy] = 0xFFFFFFFFu;
    for (int j = 1; j < kRsLen; ++j) ring_state[j] = 0u;
    *remote_n = 0u;
    window_rows_body(counts, 0u, cap, rows, gen);
  }
}

}  // namespace

int select_grid(int cap) {
  int g = (cap + 4095) / 4096;
  return g < 1 ? 1 : (g > 1024 ? 1024 : g);
}

void launch_select(const SignalCols& gc, const int* rows, const int* counts, int cap, uint32_t* blk_cnt,
                   uint32_t* blk_off, XRec* out, uint32_t* n_out, uint32_t out_cap, hipStream_t stream,
                   unsigned long long* dropped) {
  const SelArgs a{gc, rows, counts, cap};
  const int g = select_grid(cap);
  hipLaunchKernelGGL(k_sel_count, dim3(g), dim3(kSelNT), 0, stream, a, blk_cnt);
  hipLaunchKernelGGL(k_sel_scan, dim3(1), dim3(1024), 0, stream, blk_cnt, g, blk_off, n_out, out_cap, dropped);
  hipLaunchKernelGGL(k_sel_scatter, dim3(g), dim3(kSelNT), 0, stream, a, blk_off, out, out_cap);
}

void launch_select_masked(const SignalCols& gc, const int* rows, int cap, const uint32_t* blk_cnt, uint32_t* blk_off,
                          const unsigned long long* mask, int mask_stride, XRec* out, uint32_t* n_out,
                          uint32_t out_cap, hipStream_t stream, unsigned long long* dropped) {
  const int g = decode_grid(cap);  // segment 0's decode grid (its counts and masks)
  hipLaunchKernelGGL(k_sel_scan, dim3(1), dim3(1024), 0, stream, blk_cnt, g, blk_off, n_out, out_cap, dropped);
  hipLaunchKernelGGL((k_sel_scatter_mask<1024>), dim3(g), dim3(1024), 0, stream, gc, rows, cap, mask, mask_stride,
                     blk_off, out, out_cap);
}

void launch_remote_merge(const uint8_t* xrecv, size_t stride, int world, int me, SigRec* imp, uint32_t* remote_n,
                         uint32_t imp_cap, int max_rows, hipStream_t stream, unsigned long long* dropped) {
  int g = (max_rows + 255) / 256;
  g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
  hipLaunchKernelGGL(k_remote_merge, dim3(g), dim3(256), 0, stream, xrecv, stride, world, me, imp, remote_n, imp_cap,
                     dropped);
}

void launch_window_rows(const int* counts, const uint32_t* remote_n, int cap, int* rows, GenMeta* gen,
                        hipStream_t stream) {
  hipLaunchKernelGGL(k_window_rows, dim3(1), dim3(64), 0, stream, counts, remote_n, cap, rows, gen);
}

void launch_window_begin(const FillList& fl, GenMeta* gen, unsigned long long* tmax, int gens, long long halo_ns,
                         uint32_t* ring_state, uint32_t* remote_n, const int* counts, int cap, int* rows,
                         hipStream_t stream) {
  hipLaunchKernelGGL(k_window_begin, dim3(256), dim3(256), 0, stream, fl, gen, tmax, gens, halo_ns, ring_state,
                     remote_n, counts, cap, rows);
}

}  // namespace mislo
