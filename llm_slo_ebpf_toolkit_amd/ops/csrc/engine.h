// Native per-GPU window engine: the agent's executor, with no Python or PyTorch on the
// per-window path. One process drives one MI355X; window k uses buffer b = k % nb (nb = 3):
//
//   host           : cut the window (ring positions) and hand the engine the byte ranges; the
//                    host never reads or rewrites a record
//   copy stream    : DMA of the window's ring bytes straight from the (registered) rings into
//                    device block b: the BPF ring's framed records as the kernel wrote them,
//                    the user-space producers' 64-byte records, the spans, the counts
//   compute stream : [device refit from window k - nb's all-reduced statistics]
//                    graph(b): reset accumulators -> ring definitions (context rows, trace
//                    map) -> K1 decode (framed + user records) -> partition -> spans -> K2 LDS
//                    join -> finalize -> K3 MFMA posterior (+ confusion, + MFMA sufficient
//                    statistics when learning) -> pack(packet b) -> D2H of the per-incident
//                    results into pinned results b
//   comm stream    : one RCCL group over xGMI when the node has several GPUs: all-reduce(packet
//                    b), all-gather of the window's incident results (node-wide incident list),
//                    all-gather of the trace-tagged rows (merged into window k+1's imports) ->
//                    totals += packet b -> D2H(packet b, all ranks' results)
//
// Halo and imported rows: window k also joins (never counts) the rows of up to halo_windows
// earlier windows that lie within halo_ms of each later window's latest record -- kept resident
// where their own window decoded and partitioned them -- and the other GPUs' trace-tagged rows of
// window k (exchange.hip), so joins across window and GPU boundaries match.
//
// so the DMA of window k+1 and the node-wide all-reduce of window k run under the kernels of
// window k+1. The whole compute chain of a buffer is captured once into a HIP graph and
// replayed (one launch per window). Host waits use blocking-sync events (no spin: the
// agent's CPU budget, REF pkg/safety/overhead_guard.go:77-107, counts this process).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <map>
#include <tuple>
#include <vector>

#include "mislo_launch.h"
#include "mislo_packet.h"

namespace mislo {

constexpr uint32_t kCtxRows = 1u << 24;                 // device context table rows (256 MiB)
constexpr uint32_t kPodRows = 1u << 20;                 // device pod table: pod id -> svc<<16|node
constexpr uint32_t kTraceIdRows = 1u << 24;             // device trace id -> hash table (128 MiB)
constexpr int kHeadBytes = 64;                          // counts int32[16] (labels follow)

// A host byte range to DMA (a ring segment): registered memory goes straight to the device,
// anything else through the engine's pinned staging.
struct Seg {
  const void* ptr;
  size_t bytes;
};

struct EngineConfig {
  int device = 0;
  int sig_cap = 1 << 20, span_cap = 16384, group_cap = 64;
  int user_cap = 1 << 18;  // user-space (64-byte) records per window; sig_cap bounds framed + user
  int n_buffers = 3, max_ahead = 3;
  double window_ms = 2000.0, threshold = 0.7;
  int fanout = 3, group_mode = 1;
  bool use_graphs = true;
  bool device_refit = true;  // learned naive Bayes refit on the device from accumulated statistics
  double alpha = 2.0, prior_pseudo = 1.0;
  double inv_temp = 1.0, min_count = 0.0;  // refit calibration (posterior.hip k_refit_nb)
  int cap_dom = -1;                         // refit: the domain whose prior is capped (-1: none)
  double lik_ceil = 1.0;                    // refit: every likelihood capped here (models/train.py lik_ceil)
  int n_dom = 10;
  float ttft_slo_ms = 800.0f;  // per-incident SLO impact: spans with TTFT above this breach
  double halo_ms = 0.0;        // later windows also join rows this close to every later window's latest record
  int halo_windows = 3;        // earlier windows whose rows stay resident for the halo (1..3)
  int import_cap = 0;          // other GPUs' trace rows per window; 0 = none
  int xchg_cap = 0;            // trace-tagged rows each GPU exchanges per window (RCCL); 0 = none
  // group sharding of one node's stream over the node's GPUs (agent --gpus N): this GPU counts and
  // joins only its services' records and incident groups (decode.hip shard_owns); 1 = whole stream
  int shard_rank = 0, shard_world = 1;
  // split rings (agent --gpus N with per-worker rings): the producers already routed every record
  // to the ring of the worker owning its service, so the records are not filtered again here (a
  // record routed before its pod's service was known is counted where it landed, never twice);
  // spans keep the ownership filter (it also maps global groups to this GPU's local ones)
  bool split_rings = false;
};

// per-incident results of a window, in one pinned block (one D2H)
struct ResultView {
  const double* post;     // [G][16]
  const double* gconf;    // [G]
  const float* feat;      // [G][16]
  const int32_t* pred;    // [G]
  const uint32_t* evbits; // [G][16]
  const uint32_t* sli;    // [G][2]: spans, TTFT-SLO breaches
  const uint32_t* app;    // [G][2]: spans with an application retrieval time, its sum (10 us units)
  const uint32_t* late;   // [G][2]: breaches of earlier windows reported in this one (SpanMap::grp_late), spare
};

// The window's inputs: ring byte ranges (as the rings hold them) and the window metadata.
struct WindowInput {
  std::vector<Seg> kernel;  // framed BPF ring batch records (136-byte stride), in ring order
  std::vector<Seg> user;    // user-space producers' records: 64-byte EVENT or 32-byte User32
  int user_rec = 64;        // their size
  std::vector<Seg> spans;   // 64-byte SPAN records
  int n_groups = 0;
  const int32_t* labels = nullptr;  // [n_groups] ground-truth domain (replay / evaluation) or null
  int64_t bases[4] = {0, 0, 0, 0};  // epoch bases by tag
};

class WindowEngine {
 public:
  explicit WindowEngine(const EngineConfig& cfg);
  ~WindowEngine();
  WindowEngine(const WindowEngine&) = delete;
  WindowEngine& operator=(const WindowEngine&) = delete;

  const EngineConfig& config() const { return cfg_; }
  int buffers() const { return nb_; }

  // Page-lock a host range (a ring's mapping) so its bytes DMA straight to the device; false if
  // the driver refuses (those ranges then go through pinned staging).
  bool register_host(const void* ptr, size_t bytes);
  // Queue window k (in order). Returns when its DMAs and kernels are queued; the ring bytes
  // must stay untouched until h2d_done(k).
  void submit(int64_t k, const WindowInput& in, bool with_labels, bool learn);
  bool h2d_done(int64_t k);   // window k's input DMAs completed (its ring space may be freed)
  void wait_h2d(int64_t k);
  bool query(int64_t k);      // window k's results are in host memory
  void wait(int64_t k);
  const double* packet(int64_t k) const { return packet_host_[k % nb_]; }
  ResultView results(int64_t k) const;
  // device time of window k (ms): DMA start -> results in host memory, and the compute stream's share
  std::pair<float, float> window_ms(int64_t k);
  std::vector<float> copy_ms(int64_t k);  // window k's DMA time and the copy stream's idle gap before it

  void set_model_bytes(const void* bytes, size_t n);  // stream-ordered before the next window
  // device refit parameters (smoothing, prior pseudo-count, 1 / temperature, minimum labelled mass
  // of an active domain), and a refit of the model from the accumulated statistics now
  // (stream-ordered before the next window)
  void set_refit(double alpha, double prior_pseudo, double inv_temp, double min_count, int cap_dom = -1,
                 double ceil = 1.0);
  void refit_now();
  // stop (or resume) the per-window prequential refit: the model on the device stays frozen
  void set_device_refit(bool on) { cfg_.device_refit = on; }
  // Score n incidents' features [n][16] with the model on the device (the K3 posterior kernel;
  // synchronous, drains the engine first): post [n][16], pred [n], conf [n], evbits [n][16], and
  // the confusion of labels (label_code, may be null) x predictions [16][16].
  // app_cnt (optional, [n][2]): the incidents' application retrieval counts for the application
  // evidence (set_app_model)
  void score_features(const float* feat, int n, const int32_t* labels, double* post, int32_t* pred, double* conf,
                      uint32_t* evbits, uint32_t* confusion, const uint32_t* app_cnt = nullptr);
  // the application evidence model (mislo_launch.h AppModel), stream-ordered before the next window
  void set_app_model(const void* bytes, size_t n);
  // device refit: [16 x 16] Beta-prior table, optionally followed by a [16 x 16] likelihood floor
  void set_p0(const double* p0, size_t n);
  void set_pods(const uint32_t* pods, const uint32_t* svcnode, size_t n);  // pod metadata (stream-ordered)
  // other GPUs' rows for the next window, as their exchange blocks would arrive over RCCL (world
  // blocks of [24-byte header: uint32 row count | XRec rows], this rank's block skipped); the
  // next submit runs the exchange path (decode part 1, merge, part 2) with them

  void inject_remote(const void* blocks, size_t stride, int world, int me);
  void set_join_params(double window_ms, double threshold, int fanout, int group_mode);
  void init_comm(const ncclUniqueId& id, int rank, int world);
  bool has_comm() const { return comm_ != nullptr; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  // all ranks' per-incident results of window k ([world] blocks of result_bytes(); this rank's
  // alone without a communicator)
  const uint8_t* results_all(int64_t k) const { return comm_ ? res_all_host_[k % nb_] : res_host_[k % nb_]; }
  size_t result_bytes() const { return res_bytes_; }

  void totals(double* out);           // accumulated (all-reduced) packets (synchronous)
  void reset_totals();
  void stats_acc(double* out);        // the device refit's accumulated statistics (synchronous)
  // restore a checkpoint: accumulated statistics, the model image (model_bytes = 0: refit it
  // on the device from the statistics) and the folded-window count
  void restore(const double* stats, const void* model, size_t model_bytes, int64_t folded);
  void model_bytes(void* out);        // the model currently on the device (synchronous)
  void sync();
  // device-side import state (synchronous; diagnostics and tests): rows[0..1], tmax, the
  // generations (count, current slot, windows held, per-age cut-offs and rows), per buffer the
  // other-GPU row counts
  std::vector<int64_t> import_state();
  // this GPU's exchange block of the last window (header: row count | XRec rows; empty without
  // the exchange): what the all-gather delivers to the other GPUs (tests)
  std::vector<uint8_t> sent_block();
  int64_t windows_folded() const { return folded_; }
  size_t staged_bytes() const { return staged_bytes_; }
  size_t direct_bytes() const { return direct_bytes_; }
  size_t graphs() const { return graphs_.size(); }
  double host_issue_us() const { return issue_n_ ? issue_us_ / issue_n_ : 0.0; }
  // of which: blocked on back-pressure events, and issuing the window's DMAs
  double host_wait_us() const { return issue_n_ ? wait_us_ / issue_n_ : 0.0; }
  double host_dma_issue_us() const { return issue_n_ ? dma_us_ / issue_n_ : 0.0; }
  double host_launch_us() const { return issue_n_ ? launch_us_ / issue_n_ : 0.0; }  // the chain's launch
  double host_pre_us() const { return issue_n_ ? pre_us_ / issue_n_ : 0.0; }     // stream waits + refit
  double host_tail_us() const { return issue_n_ ? tail_us_ / issue_n_ : 0.0; }   // results D2H + comm stream

 private:
  // the record ownership filter's (rank, world): none with split rings (EngineConfig::split_rings)
  int rec_shard_rank() const { return cfg_.split_rings ? 0 : cfg_.shard_rank; }
  int rec_shard_world() const { return cfg_.split_rings ? 1 : cfg_.shard_world; }
  void alloc();
  void set_buffer(int b);
  void run_begin(int b, hipStream_t st);
  void run_part1(int b, hipStream_t st, bool xchg);
  void run_part2(int b, int n_groups, bool with_labels, bool learn, hipStream_t st, bool xchg);
  // the window's span side (decode, partition, probe work list, span sort) on side_, forked
  // from `st` after the accumulators are reset and joined before the probe (one-GPU chain)
  void run_span_branch(int b, hipStream_t st);
  void run_spans(int b, hipStream_t st);
  void launch_part(int part, int b, int n_groups, bool with_labels, bool learn, bool xchg);
  SignalCols sig_cols() const;
  SpanCols span_cols() const;
  bool registered(const void* p, size_t n) const;
  size_t dma(const std::vector<Seg>& segs, uint8_t* dst, size_t cap, uint8_t*& staging, size_t& st_off,
             hipStream_t st);

  EngineConfig cfg_;
  int nb_, max_ahead_;
  size_t off_kern_ = 0, off_user_ = 0, off_span_ = 0, in_bytes_ = 0;  // device input block layout
  // the BPF ring bytes a window of sig_cap rows can hold: whole batch records
  size_t kern_bytes() const { return (size_t)kRecStride * (((size_t)cfg_.sig_cap + kBatchSlots - 1) / kBatchSlots); }
  std::vector<std::pair<const uint8_t*, size_t>> registered_;
  size_t staged_bytes_ = 0, direct_bytes_ = 0;
  uint32_t *pod_sn_ = nullptr, *pod_host_ = nullptr, *ring_state_ = nullptr;
  unsigned long long* trace_hash_ = nullptr;  // kernel trace id -> hash
  uint32_t* sli_ = nullptr;
  uint32_t* app_ = nullptr;         // this buffer's [G][2] application retrieval counts (after sli_)
  uint32_t* late_ = nullptr;        // this buffer's [G][2] late breaches (after app_)
  AppModel* app_dev_ = nullptr;     // the application evidence model (device)
  // other GPUs' rows: per buffer, imported after this window's records; counts per buffer
  int n_rows_ = 0;                 // rows per generation = sig_cap + import_cap
  int gens_ = 1;                   // resident generations (1 + halo_windows with a halo)
  int* rows_ = nullptr;            // device: rows of the current window
  unsigned long long* tmax_ = nullptr;
  GenMeta* gen_ = nullptr;         // device: generation slots, halo cut-offs, time ranges
  KeyTs* g_keys_ = nullptr;        // [gens][kKeyTypes * n_rows] partition list keys
  std::vector<SigRec*> imp_;
  uint32_t *remote_n_ = nullptr, *sel_cnt_ = nullptr, *sel_off_ = nullptr;
  unsigned long long* sel_mask_ = nullptr;  // the fused selection's ballot masks (nullptr: two passes)
  int sel_stride_ = 0;
  uint8_t *xsend_ = nullptr, *xrecv_ = nullptr;
  size_t xstride_ = 0, xrecv_bytes_ = 0;
  int nblk_imp_ = 0;                    // decode blocks of the other GPUs' rows
  bool spin_ = false;
  std::vector<uint8_t> inject_;         // exchange blocks for the next window (inject_remote)
  size_t inject_stride_ = 0;
  int inject_world_ = 0, inject_me_ = 0;
  int rank_ = 0, world_ = 1;
  std::vector<uint8_t*> res_all_dev_, res_all_host_;
  std::vector<hipEvent_t> xchg_done_;
  // span branch: a second compute stream, overlapping the span side of the chain (~50 us of
  // small kernels, plus the one-workgroup probe work list) with the signal side's decode and
  // scatter, joined before the probe: the one-GPU chain only (with the exchange the window runs
  // as two graphs on the compute stream). On by default, off with MISLO_ONE_STREAM (the
  // one-queue agent) or MISLO_SPAN_STREAM=0 (profiles/r5_probe/README.md).
  hipStream_t side_ = nullptr;
  hipEvent_t ev_fork_ = nullptr, ev_sigbase_ = nullptr, ev_spans_ = nullptr;
  bool branch_ = false;
  bool xspan_ = false;  // with the exchange: window head (part 4) and span side on side_ (part 3)
  bool exchange() const { return comm_ && cfg_.xchg_cap > 0 && cfg_.import_cap > 0; }
  JoinParams jp_{};
  int nblk_sig_ = 1, nblk_span_ = 1;
  hipStream_t copy_ = nullptr, copy2_ = nullptr, compute_ = nullptr, comm_stream_ = nullptr;
  ncclComm_t comm_ = nullptr;
  ncclComm_t xcomm_ = nullptr;  // the trace-row exchange's communicator (compute stream; init_comm)
  // device buffers
  std::vector<uint8_t*> in_dev_;     // per buffer: [head | framed | user | spans]
  std::vector<uint8_t*> head_host_;  // per buffer: counts + labels (pinned)
  std::vector<uint8_t*> staging_;    // per buffer: pinned staging for unregistered ranges
  std::vector<double*> packet_dev_;
  std::vector<double*> packet_host_;
  std::vector<uint8_t*> res_dev_, res_host_;  // per buffer
  size_t res_bytes_ = 0;
  uint32_t* ctx_tab_ = nullptr;
  double *totals_ = nullptr, *stats_acc_ = nullptr, *p0_ = nullptr;
  uint8_t* model_dev_ = nullptr;
  std::vector<uint8_t*> model_host_;
  int model_slot_ = 0;
  uint8_t* g_status_ = nullptr;
  PartCodes* g_part_ = nullptr;
  uint32_t *g_part_blk_ = nullptr, *g_part_off_ = nullptr, *g_part_tot_ = nullptr, *g_part_base_ = nullptr,
           *g_items_ = nullptr;
  SigRec* g_rec_ = nullptr;
  PartCodes* s_part_ = nullptr;
  uint32_t *s_part_blk_ = nullptr, *s_part_off_ = nullptr, *s_part_tot_ = nullptr, *s_part_base_ = nullptr,
           *s_items_ = nullptr, *probe_work_ = nullptr;
  PreSpan* s_pre_ = nullptr;  // the probe's per-window sorted span lists (k_span_sort)
  SpanRec* s_rec_ = nullptr;
  unsigned long long* top3_ = nullptr;
  uint32_t* cnt_ = nullptr;
  float *attrs_ = nullptr, *conf_ = nullptr, *kernel_ms_ = nullptr;
  unsigned long long* gsum_ = nullptr;
  uint32_t* gcnt_ = nullptr;
  uint32_t *hist_ = nullptr, *status_ = nullptr, *confusion_ = nullptr;
  unsigned long long *misc_ = nullptr, *dbg_ = nullptr;
  double *stats_ = nullptr, *stats_count_ = nullptr;
  // results block views (device)
  double *post_ = nullptr, *gconf_ = nullptr;
  float* feat_ = nullptr;
  int32_t* pred_ = nullptr;
  uint32_t* evbits_ = nullptr;
  // events
  std::vector<hipEvent_t> h2d_done_, h2d_part_, head_done_, compute_done_, comm_done_;
  std::vector<hipEvent_t> t_start_, t_copy_end_, t_comp0_, t_comp1_, t_end_;
  std::map<std::tuple<int, int, bool, bool>, hipGraphExec_t> graphs_;
  std::vector<bool> warm_;
  std::vector<hipGraph_t> graph_defs_;
  int64_t submitted_ = 0, folded_ = 0;
  double issue_us_ = 0, wait_us_ = 0, dma_us_ = 0, launch_us_ = 0, pre_us_ = 0, tail_us_ = 0;
  double split_us_[4] = {0, 0, 0, 0};  // DMA issue: ring bytes, head, user records, spans

 public:
  std::vector<double> host_dma_split_us() const {
    std::vector<double> v;
    for (double x : split_us_) v.push_back(issue_n_ ? x / issue_n_ : 0.0);
    return v;
  }

 private:
  int64_t issue_n_ = 0;
};

void engine_set_tables(const Tables& t);

}  // namespace mislo
