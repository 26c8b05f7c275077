// One window's host work, end to end, into the pinned input block the engine DMAs
// (slot.h): the agent's whole per-window CPU cost lives here.
//
//   1. kernel records: RingbufConsumer compacts the BPF ring's committed EVENT16 records up to
//      the window cut straight into the block's event region (worker pool), and returns the
//      probes' definition records;
//   2. AgentTables turns the definitions into trace-map entries and context rows;
//   3. user-space producers' 64-byte records (rocprofiler-sdk tool, instrumented services; the
//      shared-memory MPSC ring) are encoded to EVENT16 behind the kernel records;
//   4. spans (the span ring fed by the OTLP receiver / services) -> SPAN20;
//   5. the new context rows go into the block's row patch, counts and labels into its head.
// REF's equivalent is one goroutine per ring decoding record by record into a channel
// (pkg/collector/ringbuf.go:91-150); here the per-event work is a compaction copy and the
// decode runs on the GPU.
#pragma once

#include <cstdint>
#include <vector>

#include "bpfring.h"
#include "ring.h"
#include "slot.h"
#include "tables.h"

namespace mislo {

struct AssembleResult {
  uint32_t n_events = 0, n_kernel = 0, n_user = 0, n_spans = 0, n_rows = 0, n_defs = 0;
  uint32_t rows_deferred = 0;      // rows that did not fit (uploaded with the next window)
  uint64_t discarded = 0, foreign = 0;
  bool busy_stop = false;
  uint64_t ring_begin = 0, ring_end = 0;
  uint64_t user_dropped = 0;       // user-ring records beyond the window's event capacity (left queued)
  size_t dma_bytes = 0;
  double host_us = 0;
};

class WindowAssembler {
 public:
  // any source may be null (no BPF ring / no user-space producers / no span ring)
  WindowAssembler(const SlotLayout& L, AgentTables* tables, RingbufConsumer* kernel, Ring* user_events, Ring* spans);
  // limits are the window cut: ring positions snapshotted when the window was closed
  // (~0 = everything available now)
  AssembleResult assemble(uint8_t* slot, const int64_t bases[4], int n_groups, const int32_t* labels,
                          uint64_t kernel_limit = ~0ull, uint64_t user_limit = ~0ull, uint64_t span_limit = ~0ull);
  const SlotLayout& layout() const { return L_; }

 private:
  SlotLayout L_;
  AgentTables* tables_;
  RingbufConsumer* kernel_;
  Ring* user_;
  Ring* spans_;
  std::vector<Rec16> defs_;
  std::vector<uint32_t> row_ids_;
  std::vector<AgentTables::Row> rows_;
};

}  // namespace mislo
