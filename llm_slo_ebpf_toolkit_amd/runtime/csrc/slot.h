// Layout of one window's input block, identical in pinned host memory (written by the
// agent's WindowAssembler) and in device memory (read by the window kernels), so a window
// crosses PCIe as ONE DMA of its used prefix:
//
//   0        counts int32[16]   [0] events, [1] spans, [2] incident groups, [3] node-local
//                               events (0 = all), [4..5] epoch base 0, [6] -, [7] span
//                               record bytes (20), [8..13] epoch bases 1-3, [14] context-row
//                               patch rows, [15] -
//   64       labels int32[group_cap]
//   sp_off   spans SPAN20[span_cap]          (fixed region, 64-aligned)
//   ev_off   events EVENT16[n_events]        (64-aligned): kernel-ring records, then host-encoded
//   ev_off + 16 n_events:
//            context-row patch: ids u32[n_rows], pad to 16, rows uint4[n_rows]
//   DMA length = ev_off + 16 n_events + row patch bytes
#pragma once

#include <cstddef>
#include <cstdint>

namespace mislo {

constexpr int kSlotCounts = 16;

struct SlotLayout {
  uint32_t group_cap, span_cap, sig_cap, row_cap;
  size_t sp_off, ev_off, bytes;
};

inline size_t round64(size_t x) { return (x + 63) & ~size_t(63); }
inline size_t round16(size_t x) { return (x + 15) & ~size_t(15); }

inline SlotLayout slot_layout(uint32_t group_cap, uint32_t span_cap, uint32_t sig_cap, uint32_t row_cap) {
  SlotLayout L{group_cap, span_cap, sig_cap, row_cap, 0, 0, 0};
  L.sp_off = round64(64 + 4 * (size_t)group_cap);
  L.ev_off = round64(L.sp_off + 20 * (size_t)span_cap);
  L.bytes = round64(L.ev_off + 16 * (size_t)sig_cap + round16(4 * (size_t)row_cap) + 16 * (size_t)row_cap);
  return L;
}

// bytes of the row patch that follows n_events events
inline size_t row_patch_bytes(uint32_t n_rows) { return round16(4 * (size_t)n_rows) + 16 * (size_t)n_rows; }

inline size_t slot_dma_bytes(const SlotLayout& L, uint32_t n_events, uint32_t n_rows) {
  return L.ev_off + 16 * (size_t)n_events + (n_rows ? row_patch_bytes(n_rows) : 0);
}

}  // namespace mislo
