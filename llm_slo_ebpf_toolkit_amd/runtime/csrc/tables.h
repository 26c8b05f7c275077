// The agent's host-side id tables: everything the GPU needs besides the ring bytes.
//
//   * device context table (2^24 rows of {pod, pid, conn32, svc<<16|node}, HBM-resident for the
//     agent's lifetime): rows 1 .. 2^23 - 1 are the kernel's (defined by CTX definition records
//     in the ring, svc|node filled in from the agent's pod metadata), rows 2^23 .. 2^24 - 1 the
//     host encoder's (user-space producers' records and spans). New rows of a window are handed
//     out as an (id, row) patch the window's kernels scatter into the table before decoding;
//   * trace map: trace hash -> trace id, fed by the kernel's TRACE definitions (ids < 2^24) and
//     extended by the host encoder for hashes the kernel has not seen (ids >= 2^24), so spans
//     and events share one id space. Entries unused for two windows expire;
//   * the host encoder: 64-byte EVENT records from user-space producers (the rocprofiler-sdk
//     tool library, instrumented services) -> EVENT16 against the window's epoch bases, and
//     spans -> SPAN20. Exhausted host id ranges wrap (rows are rewritten as ids are reused)
//     instead of failing, so a long-running agent never stops on id exhaustion.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <vector>

#include "bpfring.h"
#include "records.h"

namespace mislo {

class AgentTables {
 public:
  using Row = std::array<uint32_t, 4>;
  explicit AgentTables(const int8_t* shift256);

  // ---- metadata ----
  void set_pod(uint32_t pod, uint32_t svcnode);  // re-queues the pod's kernel context rows if it changed
  uint32_t pod_svcnode(uint32_t pod) const { return pod < pod_sn_.size() ? pod_sn_[pod] : 0u; }

  // ---- kernel definitions (one window's side list from RingbufConsumer) ----
  void apply_defs(const Rec16* defs, size_t n);

  // ---- host encoder ----
  // 64-byte records -> EVENT16 (ts offset from the latest of bases[0..3] at or below ts, tagged
  // with its index; bases[tag] == 0 entries are unused). Returns n.
  size_t encode_events(const EventRec* ev, size_t n, Rec16* out, const int64_t bases[4]);
  void encode_spans(const SpanRec64* sp, size_t n, Span20* out);
  // per incident group, spans seen since the last take and how many breached the TTFT SLO
  // (ttft_ms > threshold): the window's SLO impact (burn rate) per incident
  void set_sli_threshold(float ttft_ms) { sli_ttft_ms_ = ttft_ms; }
  size_t take_group_sli(uint32_t* out_n, uint32_t* out_breach, size_t groups);
  uint32_t trace_id(uint64_t hash);       // lookup or host-assign
  uint32_t host_ctx(uint32_t pod, uint32_t pid, uint32_t c32, uint32_t sn);

  // ---- per-window hand-off ----
  // moves up to `cap` pending rows out (ids[i], rows[i]); returns how many
  size_t take_rows(uint32_t* ids, Row* rows, size_t cap);
  size_t pending_rows() const { return pending_.size() - pending_head_; }
  void end_window();

  size_t n_kernel_ctx() const { return kernel_rows_.size(); }
  size_t n_host_ctx() const { return host_size_; }
  size_t n_traces() const { return tr_size_; }
  uint64_t host_ctx_wraps() const { return host_wraps_; }
  uint64_t bad_defs() const { return bad_defs_; }

 private:
  void queue_row(uint32_t id, const Row& r);
  void trace_put(uint64_t hash, uint32_t id);
  void trace_rehash(size_t cap, uint32_t min_gen);
  void host_reset();

  int8_t shift_[256];
  std::vector<uint32_t> pod_sn_;
  std::vector<Row> kernel_rows_;  // index = kernel ctx id (svc|node column as last uploaded)
  // host contexts: open addressing, key (pod, pid, c32, sn) stored in the slot
  struct HSlot {
    uint32_t pod, pid, c32, sn, id;  // id 0 = empty
  };
  std::vector<HSlot> host_;
  size_t host_mask_ = 0, host_size_ = 0;
  uint32_t host_next_ = kKernelCtxLimit;
  uint64_t host_wraps_ = 0;
  // traces: open addressing, (hash, id, generation)
  struct TSlot {
    uint64_t key;
    uint32_t id, gen;
  };
  std::vector<TSlot> tr_;
  size_t tr_mask_ = 0, tr_size_ = 0;
  uint32_t tr_next_ = kKernelTraceLimit;
  uint32_t gen_ = 1;
  std::vector<std::pair<uint32_t, Row>> pending_;
  float sli_ttft_ms_ = 800.0f;
  std::vector<uint32_t> grp_n_, grp_breach_;
  size_t pending_head_ = 0;
  uint64_t bad_defs_ = 0;
};

}  // namespace mislo
