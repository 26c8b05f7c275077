// Window-to-window and GPU-to-GPU record exchange of the native engine.
//
//   halo   : the decoded rows of window k whose timestamps lie within the join window of the
//            window's latest local record are carried into window k+1 as imported rows, so a
//            span early in window k+1 still finds the signals recorded just before the cut
//            (REF correlates against a continuous 2 s buffer, pkg/correlation/dns.go:12).
//   remote : each GPU's trace-tagged local rows of window k at warn level or above (the
//            evidence; identity dropped: only their trace hash can join) are all-gathered over
//            RCCL on the comm stream as 32-byte XRecs and imported into window k+1 on every other
//            GPU, so a request traced across nodes joins the elevated signals of every node that
//            saw it.
//
// Both are stable stream compactions (count -> exclusive scan -> ordered scatter), so the
// imported rows, and with them the join's tie-breaks by row index, are deterministic.
#include "mislo_common.h"
#include "mislo_launch.h"

namespace mislo {

namespace {

constexpr int kSelNT = 256;

struct SelArgs {
  const SigRec* rec;
  const uint8_t* status;  // per row: 0 ok, 1 warn, 2 error
  const int* rows;      // rows[0] = rows of the window (local + imported)
  const int* counts;    // counts[0] = local rows
  int cap;
  int mode;             // kSelHalo | kSelTrace
  const unsigned long long* tmax;
  long long halo_ns;
};

__device__ __forceinline__ int sel_end(const SelArgs& a) {
  const int n = min(a.rows[0], a.cap);
  return a.mode == kSelTrace ? min(a.counts[0], n) : n;
}

__device__ __forceinline__ bool selected(const SelArgs& a, const SigRec& r, int i, unsigned long long tmax) {
  if (r.slot == kNoSlot || r.ts == 0) return false;
  if (a.mode == kSelTrace) return r.tr != 0 && a.status[i] >= 1;
  return tmax != 0 && r.ts >= (long long)tmax - a.halo_ns;
}

// per-block counts of selected rows (fixed grid; block b owns a contiguous chunk)
__global__ __launch_bounds__(kSelNT) void k_sel_count(SelArgs a, uint32_t* __restrict__ blk_cnt) {
  const int n = sel_end(a);
  const unsigned long long tmax = *a.tmax;
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);
  uint32_t c = 0;
  for (int i = beg + threadIdx.x; i < end; i += kSelNT) c += selected(a, a.rec[i], i, tmax) ? 1u : 0u;
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

// exclusive scan of <= 1024 block counts; total (clamped to the output capacity) -> *n_out
__global__ __launch_bounds__(1024) void k_sel_scan(const uint32_t* __restrict__ blk_cnt, int nblk,
                                                  uint32_t* __restrict__ blk_off, uint32_t* __restrict__ n_out,
                                                  uint32_t out_cap) {
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
  if (t == 1023) *n_out = min(s[1023], out_cap);
}

// ordered scatter: block offset + wave offsets + in-wave ballot rank; full SigRec rows (halo)
// or 32-byte exchange rows (XRec: no identity)
__global__ __launch_bounds__(kSelNT) void k_sel_scatter(SelArgs a, const uint32_t* __restrict__ blk_off,
                                                        void* __restrict__ out, uint32_t out_cap, int xrec) {
  const int n = sel_end(a);
  const unsigned long long tmax = *a.tmax;
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
      r = a.rec[i];
      s = selected(a, r, i, tmax);
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
      if (dst < out_cap) {
        if (xrec)  // a remote row joins through its trace hash only
          static_cast<XRec*>(out)[dst] = XRec{r.ts, r.tr, r.val, r.slot, 0, 0};
        else
          static_cast<SigRec*>(out)[dst] = r;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int q = 0; q < kSelNT / 64; ++q) t += s_w[q];
      s_base += t;
    }
  }
}

// other GPUs' exchanged rows (each rank's block: a 32-byte header holding its row count, then
// XRec rows) appended after this window's halo rows as identity-free SigRecs, in rank order
__global__ __launch_bounds__(256) void k_remote_merge(const uint8_t* __restrict__ xrecv, size_t stride, int world,
                                                      int me, SigRec* __restrict__ imp,
                                                      const uint32_t* __restrict__ halo_n,
                                                      uint32_t* __restrict__ remote_n, uint32_t imp_cap) {
  const uint32_t h = *halo_n;
  uint32_t off = h;
  for (int r = 0; r < world; ++r) {
    if (r == me) continue;
    const uint8_t* blk = xrecv + (size_t)r * stride;
    const uint32_t c = min(*reinterpret_cast<const uint32_t*>(blk), (uint32_t)((stride - sizeof(XRec)) / sizeof(XRec)));
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
  if (blockIdx.x == 0 && threadIdx.x == 0) *remote_n = (off < imp_cap ? off : imp_cap) - h;
}

// rows of the window: rows[0] = local records + the imported halo (decode segment 0),
// rows[1] = rows[0] + other GPUs' rows (segment 1)
__global__ void k_window_rows(const int* __restrict__ counts, const uint32_t* __restrict__ halo_n,
                              const uint32_t* __restrict__ remote_n, int cap, int* __restrict__ rows) {
  if (threadIdx.x == 0) {
    const long long a = (long long)counts[0] + *halo_n;
    const long long r0 = a < cap ? a : cap;
    const long long b = r0 + *remote_n;
    rows[0] = (int)r0;
    rows[1] = (int)(b < cap ? b : cap);
  }
}

}  // namespace

int select_grid(int cap) {
  int g = (cap + 4095) / 4096;
  return g < 1 ? 1 : (g > 1024 ? 1024 : g);
}

void launch_select(const SigRec* rec, const uint8_t* status, const int* rows, const int* counts, int cap, int mode,
                   const unsigned long long* tmax, long long halo_ns, uint32_t* blk_cnt, uint32_t* blk_off, void* out,
                   uint32_t* n_out, uint32_t out_cap, bool xrec, hipStream_t stream) {
  const SelArgs a{rec, status, rows, counts, cap, mode, tmax, halo_ns};
  const int g = select_grid(cap);
  hipLaunchKernelGGL(k_sel_count, dim3(g), dim3(kSelNT), 0, stream, a, blk_cnt);
  hipLaunchKernelGGL(k_sel_scan, dim3(1), dim3(1024), 0, stream, blk_cnt, g, blk_off, n_out, out_cap);
  hipLaunchKernelGGL(k_sel_scatter, dim3(g), dim3(kSelNT), 0, stream, a, blk_off, out, out_cap, xrec ? 1 : 0);
}

void launch_remote_merge(const uint8_t* xrecv, size_t stride, int world, int me, SigRec* imp, const uint32_t* halo_n,
                         uint32_t* remote_n, uint32_t imp_cap, int max_rows, hipStream_t stream) {
  int g = (max_rows + 255) / 256;
  g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
  hipLaunchKernelGGL(k_remote_merge, dim3(g), dim3(256), 0, stream, xrecv, stride, world, me, imp, halo_n, remote_n,
                     imp_cap);
}

void launch_window_rows(const int* counts, const uint32_t* halo_n, const uint32_t* remote_n, int cap, int* rows,
                        hipStream_t stream) {
  hipLaunchKernelGGL(k_window_rows, dim3(1), dim3(64), 0, stream, counts, halo_n, remote_n, cap, rows);
}

}  // namespace mislo
