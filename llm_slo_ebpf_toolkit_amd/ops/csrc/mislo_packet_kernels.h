// The packet's device kernels (internal linkage: include in ONE translation unit per module).
#pragma once

#include "mislo_packet.h"

namespace mislo {
namespace {

__global__ __launch_bounds__(256) void k_fill(FillList fl) {
  for (int q = 0; q < fl.count; ++q) {
    const FillSeg sg = fl.seg[q];
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < sg.n; i += gridDim.x * 256) sg.ptr[i] = sg.value;
  }
}

// packet element i (< kPacketLen) from the window's accumulators; ring (RingState) may be null
__device__ __forceinline__ double packet_value(int i, const uint32_t* hist, const uint32_t* status,
                                               const unsigned long long* misc, const unsigned long long* dbg,
                                               const uint32_t* confusion, const double* stats, const double* count,
                                               const uint32_t* ring) {
  int o = 0;
  if (i < kPacketHist) return hist[i];
  o += kPacketHist;
  if (i < o + kPacketStatus) return status[i - o];
  o += kPacketStatus;
  if (i < o + kPacketMisc) return (double)misc[i - o];
  o += kPacketMisc;
  if (i < o + kPacketDbg) return (double)dbg[i - o];
  o += kPacketDbg;
  if (i < o + kPacketConf) return confusion[i - o];
  o += kPacketConf;
  if (i < o + kPacketStats) return stats[i - o];
  o += kPacketStats;
  if (i < o + kPacketCount) return count[i - o];
  o += kPacketCount;
  const uint32_t v = ring ? ring[i - o] : (i - o == kRsFirstBusy ? 0xFFFFFFFFu : 0u);
  return (i - o == kRsFirstBusy && v == 0xFFFFFFFFu) ? -1.0 : (double)v;  // -1: no busy record
}

// accumulators -> packet (f64), one element per thread
__global__ void k_pack(const uint32_t* hist, const uint32_t* status, const unsigned long long* misc,
                       const unsigned long long* dbg, const uint32_t* confusion, const double* stats,
                       const double* count, const uint32_t* ring, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < kPacketLen) out[i] = packet_value(i, hist, status, misc, dbg, confusion, stats, count, ring);
}

}  // namespace
}  // namespace mislo
