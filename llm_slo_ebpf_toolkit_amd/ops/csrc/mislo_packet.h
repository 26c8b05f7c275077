// The window packet: everything a window contributes to the node-wide totals, packed in f64 so
// ONE all-reduce (RCCL over xGMI) fuses every GPU's counters per window. One layout for every
// engine (engine.hip's WindowEngine and the kernel unit-test harness in bindings.cpp):
//   [hist 16x16 | status 16x3 | misc 2+16 | dbg 8 | confusion 16x16 | stats 32x32 | count 16 | ring 8]
// pipeline/window.py PACKET_LAYOUT mirrors it (checked against the module's PACKET_LAYOUT).
#pragma once

#include "mislo_common.h"

namespace mislo {

constexpr int kPacketHist = kSlots * kBuckets;          // 256
constexpr int kPacketStatus = kSlots * 3;               // 48
constexpr int kPacketMisc = 2 + kSlots;                 // unsupported, zero-ts, per-slot value sums (milli)
constexpr int kPacketDbg = 8;
// dbg: [0] candidates [1] low confidence [2] overlap [3] fanout dropped [4] spans enriched, then the
// multi-GPU exchange's losses: [5] trace rows selected beyond the exchange capacity (or the sent
// block size), [6] other GPUs' rows beyond the import capacity
constexpr int kDbgXchgDropped = 5, kDbgImportDropped = 6;
constexpr int kPacketConf = kMaxDomains * kMaxDomains;  // 256
constexpr int kPacketStats = 32 * 32;                   // 1024
constexpr int kPacketCount = kMaxDomains;               // 16
constexpr int kPacketRing = kRsLen;                     // ring accounting (RingState); per GPU, never reduced
constexpr int kPacketLen =
    kPacketHist + kPacketStatus + kPacketMisc + kPacketDbg + kPacketConf + kPacketStats + kPacketCount + kPacketRing;
constexpr int kStatsOff = kPacketHist + kPacketStatus + kPacketMisc + kPacketDbg + kPacketConf;
constexpr int kStatsLen = kPacketStats + kPacketCount;  // accumulated-statistics vector (f64[1040])

// One launch that zero/poison-fills every per-window accumulator (instead of a hipMemsetAsync
// per buffer: each is a fill kernel plus launch overhead on gfx950).
struct FillSeg {
  uint32_t* ptr;
  uint32_t n;  // 32-bit words
  uint32_t value;
};
constexpr int kMaxFill = 14;
struct FillList {
  FillSeg seg[kMaxFill];
  int count;
};

}  // namespace mislo
