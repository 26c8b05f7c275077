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

// accumulators -> packet (f64), one element per thread; ring (RingState) may be null
__global__ void k_pack(const uint32_t* hist, const uint32_t* status, const unsigned long long* misc,
                       const unsigned long long* dbg, const uint32_t* confusion, const double* stats,
                       const double* count, const uint32_t* ring, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int o = 0;
  if (i < kPacketHist) { out[i] = hist[i]; return; }
  o += kPacketHist;
  if (i < o + kPacketStatus) { out[i] = status[i - o]; return; }
  o += kPacketStatus;
  if (i < o + kPacketMisc) { out[i] = (double)misc[i - o]; return; }
  o += kPacketMisc;
  if (i < o + kPacketDbg) { out[i] = (double)dbg[i - o]; return; }
  o += kPacketDbg;
  if (i < o + kPacketConf) { out[i] = confusion[i - o]; return; }
  o += kPacketConf;
  if (i < o + kPacketStats) { out[i] = stats[i - o]; return; }
  o += kPacketStats;
  if (i < o + kPacketCount) { out[i] = count[i - o]; return; }
  o += kPacketCount;
  if (i < o + kPacketRing) {
    const uint32_t v = ring ? ring[i - o] : (i - o == kRsFirstBusy ? 0xFFFFFFFFu : 0u);
    out[i] = (i - o == kRsFirstBusy && v == 0xFFFFFFFFu) ? -1.0 : (double)v;  // -1: no busy record
    return;
  }
}

}  // namespace
}  // namespace mislo
