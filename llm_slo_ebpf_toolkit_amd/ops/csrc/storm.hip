// K6: batched retry-storm windowed counts (REF pkg/correlation/retry_storm.go:46-110).
//
// REF keeps, per pod, the retransmit timestamps of the last `window` (10 s) and reports a
// storm when Record() leaves >= threshold (5) of them. For a batch whose events are
// ordered by (pod, ts) -- the arrival order of one pod's retransmits -- Record(e_i) keeps
// exactly the events j <= i of the same pod with ts_j >= ts_i - window (the prune drops
// the leading run strictly before the cutoff). So count_i = i - lower_bound(cutoff) + 1
// inside the pod's segment: two binary searches per event, no atomics, no state.
#include "mislo_launch.h"

namespace mislo {

template <int NT>
__global__ __launch_bounds__(NT) void k_storm_counts(const uint64_t* __restrict__ keys,
                                                     const int64_t* __restrict__ ts, int n, int64_t window_ns,
                                                     uint32_t threshold, uint32_t* __restrict__ counts,
                                                     unsigned long long* __restrict__ n_storm) {
  const int i = blockIdx.x * NT + threadIdx.x;
  uint32_t storm = 0;
  if (i < n) {
    const uint64_t k = keys[i];
    int lo = 0, hi = i;  // first index with key == k
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (keys[m] < k) lo = m + 1; else hi = m;
    }
    const int64_t cutoff = ts[i] - window_ns;
    hi = i;  // first index in [seg, i] with ts >= cutoff
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (ts[m] < cutoff) lo = m + 1; else hi = m;
    }
    const uint32_t c = (uint32_t)(i - lo + 1);
    counts[i] = c;
    storm = c >= threshold;
  }
  // wave-aggregated storm tally
  for (int off = 32; off > 0; off >>= 1) storm += __shfl_xor(storm, off);
  if ((threadIdx.x & 63) == 0 && storm) atomicAdd(n_storm, (unsigned long long)storm);
}

void launch_storm_counts(const uint64_t* keys, const int64_t* ts, int n, int64_t window_ns, uint32_t threshold,
                         uint32_t* counts, unsigned long long* n_storm, hipStream_t stream) {
  constexpr int NT = 256;
  if (n <= 0) return;
  hipLaunchKernelGGL((k_storm_counts<NT>), dim3((n + NT - 1) / NT), dim3(NT), 0, stream, keys, ts, n, window_ns,
                     threshold, counts, n_storm);
}

}  // namespace mislo
