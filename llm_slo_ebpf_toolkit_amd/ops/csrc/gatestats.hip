// K5: release-gate statistics on the MI355X (REF pkg/releasegate/gate.go:816-946).
//
// k_boot_quantile: one workgroup per (bootstrap iteration, sample set). Instead of
// materialising and sorting each resample, the workgroup draws n counter-based indices
// into an LDS multiplicity histogram over the *pre-sorted* sample, prefix-scans it, and
// reads the q-quantile's two order statistics straight out of the scan: O(n) per
// iteration, no sort, no global traffic except the sorted sample (L2 resident).
// Index j of iteration it of set s is  splitmix64(seed') over the counter
// (s << 63 | it << 32 | j)  -- ops/gatestats.py reproduces the stream in numpy, so the
// CPU and GPU gates compute the same confidence interval bit for bit.
//
// k_rank_counts: Mann-Whitney ranks with ties and Cliff's delta without a sort: for every
// element, counts of (all < v), (all == v), (y < v), (y > v) over LDS-staged tiles.
#include "mislo_launch.h"

namespace mislo {

constexpr int kBootMaxN = 16384;  // 64 KiB LDS multiplicity histogram per workgroup

__device__ __forceinline__ uint32_t boot_index(uint64_t seed_mix, uint32_t set, uint32_t it, uint32_t j,
                                               uint32_t n) {
  const uint64_t ctr = ((uint64_t)set << 63) | ((uint64_t)it << 32) | (uint64_t)j;
  const uint64_t x = splitmix64(ctr ^ seed_mix);
  return (uint32_t)(((x >> 32) * (uint64_t)n) >> 32);
}

template <int NT>
__global__ __launch_bounds__(NT) void k_boot_quantile(const double* __restrict__ sorted_c, int nc,
                                                      const double* __restrict__ sorted_b, int nb, double q,
                                                      int iters, uint64_t seed_mix, double* __restrict__ out) {
  __shared__ uint32_t s_cnt[kBootMaxN];
  __shared__ uint32_t s_wsum[NT / 64];
  __shared__ double s_val[2];
  const int it = blockIdx.x;
  const int set = blockIdx.y;
  const double* v = set == 0 ? sorted_c : sorted_b;
  const int n = set == 0 ? nc : nb;
  const int tid = threadIdx.x;
  for (int i = tid; i < n; i += NT) s_cnt[i] = 0;
  __syncthreads();
  for (int j = tid; j < n; j += NT) atomicAdd(&s_cnt[boot_index(seed_mix, set, it, j, n)], 1u);
  __syncthreads();

  // contiguous chunk per thread -> exclusive prefix of chunk sums (wave scan + LDS)
  const int C = (n + NT - 1) / NT;
  const int beg = min(n, tid * C), end = min(n, beg + C);
  uint32_t local = 0;
  for (int i = beg; i < end; ++i) local += s_cnt[i];
  uint32_t incl = local;
  const int lane = tid & 63, wave = tid >> 6;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off);
    if (lane >= off) incl += y;
  }
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  uint32_t base = 0;
  for (int w = 0; w < wave; ++w) base += s_wsum[w];
  uint32_t run = base + incl - local;  // exclusive prefix at chunk start

  double pos = q * (double)(n - 1);
  asm volatile("" : "+v"(pos));  // keep the product rounded (no fma into pos - flo)
  const double flo = floor(pos), fhi = ceil(pos);
  const uint32_t r_lo = (uint32_t)flo, r_hi = (uint32_t)fhi;
  for (int i = beg; i < end; ++i) {
    const uint32_t c = s_cnt[i];
    if (c) {
      if (r_lo >= run && r_lo < run + c) s_val[0] = v[i];
      if (r_hi >= run && r_hi < run + c) s_val[1] = v[i];
    }
    run += c;
  }
  __syncthreads();
  if (tid == 0) {
    double r;
    if (n == 1 || r_lo == r_hi) {
      r = s_val[0];
    } else {
      const double f = pos - flo;
      // Round each product separately (numpy's  s_lo * (1 - f) + s_hi * f): the empty asm
      // makes the products opaque so the backend cannot fuse them into v_fmac_f64.
      double a = s_val[0] * (1.0 - f), b = s_val[1] * f;
      asm volatile("" : "+v"(a), "+v"(b));
      r = a + b;
    }
    out[(size_t)set * iters + it] = r;
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_rank_counts(const double* __restrict__ vals, int n_all, int nx,
                                                    uint32_t* __restrict__ out) {
  __shared__ double s_v[NT];
  const int i = blockIdx.x * NT + threadIdx.x;
  const double v = i < n_all ? vals[i] : 0.0;
  uint32_t lt_all = 0, eq_all = 0, lt_y = 0, gt_y = 0;
  for (int t0 = 0; t0 < n_all; t0 += NT) {
    const int k = t0 + threadIdx.x;
    s_v[threadIdx.x] = k < n_all ? vals[k] : 0.0;
    __syncthreads();
    const int m = min(NT, n_all - t0);
#pragma unroll 8
    for (int u = 0; u < m; ++u) {
      const double w = s_v[u];
      const bool is_y = (t0 + u) >= nx;
      const uint32_t lt = w < v, eq = w == v, gt = w > v;
      lt_all += lt;
      eq_all += eq;
      lt_y += is_y ? lt : 0u;
      gt_y += is_y ? gt : 0u;
    }
    __syncthreads();
  }
  if (i < n_all) {
    out[i] = lt_all;
    out[n_all + i] = eq_all;
    out[2 * n_all + i] = lt_y;
    out[3 * n_all + i] = gt_y;
  }
}

int boot_max_n() { return kBootMaxN; }

void launch_boot_quantile(const double* sorted_c, int nc, const double* sorted_b, int nb, double q, int iters,
                          uint64_t seed, double* out, hipStream_t stream) {
  constexpr int NT = 256;
  hipLaunchKernelGGL((k_boot_quantile<NT>), dim3(iters, 2), dim3(NT), 0, stream, sorted_c, nc, sorted_b, nb, q,
                     iters, splitmix64(seed), out);
}

void launch_rank_counts(const double* vals, int n_all, int nx, uint32_t* out, hipStream_t stream) {
  constexpr int NT = 256;
  hipLaunchKernelGGL((k_rank_counts<NT>), dim3((n_all + NT - 1) / NT), dim3(NT), 0, stream, vals, n_all, nx, out);
}

}  // namespace mislo
