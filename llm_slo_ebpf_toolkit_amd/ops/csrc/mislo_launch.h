// Host-side launch API of the MI355X engine kernels (plain pointers + hipStream_t), so the
// torch bindings, the native agent runtime and the C++ tests can all drive them.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mislo_common.h"
#include "mislo_packet.h"

namespace mislo {

// Attribution model in linear-logit form (models/bayes.py LinearPosteriorModel), resident
// in device memory (too large for kernel arguments).
struct PosteriorModel {
  double w[kSlots][kMaxDomains];  // [slot][domain]
  double bias[kMaxDomains];       // -inf = inactive domain
  double mean[kSlots];            // continuous mode centring
  double nominal[kSlots];         // continuous mode imputation for absent signals
  float thr[kSlots];              // elevated thresholds
  uint32_t dom_mask[kMaxDomains]; // per domain: slots with P(elevated|d) >= 0.5
  uint32_t table_mask;            // slots known to the model (binary mode)
  int32_t mode;                   // 0 binary evidence, 1 continuous (log1p) features
  // 2-fault hypotheses (models/bayes.py with_pairs): pair h = {pair_a[h], pair_b[h]} is one
  // more logit column; post[] then holds each domain's marginal P(d in the incident)
  int32_t n_pairs;                // 0 = single-fault posterior
  double pair_rho;                // prior mass of the pairs (the device refit rebuilds them)
  double w2[kSlots][kMaxPairs];
  double bias2[kMaxPairs];        // -inf = inactive pair
  uint8_t pair_a[kMaxPairs];
  uint8_t pair_b[kMaxPairs];
};

// Application evidence (models/bayes.py AppEvidence): one more binary signal next to the 16 slots,
// the incident group's retrieval time that the kernel signals do not account for -- REF's
// DecomposeRetrieval (ebpfcorrelator/correlator.go:179-194) at group level: the mean application
// retrieval time of the group's spans (SpanMap::grp_app) minus the kernel-attributed share, the
// group's mean joined dns + connect + TLS latency (feature slots 0, 3, 5). A group without an
// application breakdown contributes nothing (the signal is summed out, so REF's 55 rows score
// exactly as before); otherwise elevated = residual >= thr_ms adds w[d] and present adds b[d].
constexpr int kAppBit = 16;  // its evidence bit in evbits (bits 0-15: the signal slots)
struct AppModel {
  double w[kMaxDomains];   // (log P(e|d) - log P(!e|d)) / T
  double b[kMaxDomains];   // log P(!e|d) / T
  double w2[kMaxPairs];    // the 2-fault columns' noisy-OR terms
  double b2[kMaxPairs];
  double thr_ms;           // elevated threshold of the residual (ms)
  uint32_t dom_mask;       // domains with P(e|d) >= 0.5 (evidence)
  int32_t on;              // 0: the channel is off
};

// decode.hip
void set_tables(const Tables* host_tables);
int decode_grid(int cap);
void launch_decode_events(const void* ev, const int* n_dev, int cap, const SignalCols& cols, uint32_t* hist,
                          uint32_t* status_cnt, uint32_t* part_cnt, unsigned long long* misc, hipStream_t stream);
// EVENT16 records; ctx_tab = device context table (n_ctx rows of uint4)
void launch_decode_wire(const void* ev, const int* n_dev, int cap, const uint32_t* ctx_tab, int n_ctx,
                        const SignalCols& cols, uint32_t* hist, uint32_t* status_cnt, uint32_t* part_cnt,
                        unsigned long long* misc, hipStream_t stream);
void launch_decode_ref(const void* ev, const int* n_dev, int cap, uint32_t pod, uint32_t svcnode, uint64_t trace_h,
                       const SignalCols& cols, uint32_t* hist, uint32_t* status_cnt, uint32_t* part_cnt,
                       unsigned long long* misc, hipStream_t stream);
// spans: SPAN20 (counts[7] == 20) or 64-byte SPAN; sm (optional, native engine): fold
// connections to conn32 (the context rows' connection identity), count per-group TTFT SLO
// breaches
struct SpanMap {
  int native;            // 1: native engine spans (conn32 connections)
  uint32_t* grp_sli;     // [n_groups][2]: spans, TTFT > slo
  int n_groups;
  float ttft_slo_ms;
  int sh_rank = 0, sh_world = 1;  // group sharding: this GPU keeps groups g % sh_world == sh_rank as g / sh_world
  GenMeta* gen = nullptr;         // receives the spans' time range (probe pruning of older generations)
  // [n_groups][2]: spans carrying an application retrieval time (Span::retr_ms > 0), and the sum
  // of those times in kAppUnitsPerMs units (exact integers: order-free, all-reducible)
  uint32_t* grp_app = nullptr;
  // [n_groups][2]: breaching spans flagged late (Span::flags kSpanLate: the SLO deadline passed before
  // the agent's previous cut), counted here instead of in grp_sli -- the host credits them to the
  // earlier window their breach belongs to; [2g + 1] is spare
  uint32_t* grp_late = nullptr;
};
constexpr double kAppUnitsPerMs = 100.0;  // 10 us: a u32 group sum holds 42,949 s of retrieval per window
void launch_decode_spans(const void* sp, const int* n_dev, int cap, const SpanCols& cols, uint32_t* part_cnt,
                         const uint32_t* ctx_tab, int n_ctx, hipStream_t stream, const SpanMap* sm = nullptr);
// native engine window: framed BPF ring records (counts[15] of them) + 64-byte user records
void launch_ring_defs(const uint8_t* framed, const int* n_dev, int cap, uint32_t* ctx_tab, uint32_t ctx_rows,
                      const uint32_t* pod_sn, uint32_t n_pods, const TraceIds& tt, uint32_t* ring_state,
                      hipStream_t stream);
// rows [0, counts[15]) framed, [counts[15], counts[0]) user records, then imported rows (SigRec,
// imp[i - counts[0]]) that join but are not counted: segment 0 decodes rows [0, rows[0]) (the
// records + the previous window's halo), segment 1 rows [rows[0], rows[1]) (other GPUs' rows)
// with `grid` blocks whose partition counts start at block row `blk_base`; tmax (u64) receives
// the window's latest local timestamp; user-space rows are 64-byte EVENTs or, with counts[6]
// == 32, User32 records whose svc|node comes from the pod table
void launch_decode_window(const uint8_t* framed, const void* user, const int* n_dev, const int* rows, int cap,
                          const SigRec* imp, const uint32_t* ctx_tab, int n_ctx, const TraceIds& tt,
                          uint32_t* ring_state, unsigned long long* tmax, const uint32_t* pod_sn, uint32_t n_pods,
                          const SignalCols& cols, uint32_t* hist, uint32_t* status_cnt, uint32_t* part_cnt,
                          unsigned long long* misc, hipStream_t stream, int seg = 0, int grid = 0, int blk_base = 0,
                          int sh_rank = 0, int sh_world = 1, uint32_t* sel_cnt = nullptr,
                          unsigned long long* sel_mask = nullptr, int sel_stride = 0);
// ballot masks per decode block of `cap` rows (the fused selection's mask stride)
int decode_sel_stride(int cap);

// exchange.hip: the trace-tagged rows of the GPU exchange, the other GPUs' rows, the generations
int select_grid(int cap);
// 24-byte exchange row: what another GPU needs to join a row by its trace hash (no padding:
// the all-gather moves world x (1 + xchg_cap) of them per window)
struct XRec {
  int64_t ts;
  uint64_t tr;
  float val;
  uint32_t slot;
};
static_assert(sizeof(XRec) == 24, "exchange rows are 24 bytes");
// the current generation's warn-level trace-tagged local rows -> out (stable order), count -> n_out
// dropped (optional): rows over out_cap are added to it (the packet's dbg[kDbgXchgDropped])
void launch_select(const SignalCols& gc, const int* rows, const int* counts, int cap, uint32_t* blk_cnt,
                   uint32_t* blk_off, XRec* out, uint32_t* n_out, uint32_t out_cap, hipStream_t stream,
                   unsigned long long* dropped = nullptr);
// the same selection from the counts and ballot masks segment 0's decode left (sel_cnt /
// sel_mask): scan, then an ordered scatter that reads only the selected rows
void launch_select_masked(const SignalCols& gc, const int* rows, int cap, const uint32_t* blk_cnt, uint32_t* blk_off,
                          const unsigned long long* mask, int mask_stride, XRec* out, uint32_t* n_out,
                          uint32_t out_cap, hipStream_t stream, unsigned long long* dropped = nullptr);
// dropped (optional, [2]): rows beyond a block's sent size / beyond imp_cap (dbg[kDbgXchgDropped],
// dbg[kDbgImportDropped])
void launch_remote_merge(const uint8_t* xrecv, size_t stride, int world, int me, SigRec* imp, uint32_t* remote_n,
                         uint32_t imp_cap, int max_rows, hipStream_t stream, unsigned long long* dropped = nullptr);
void launch_window_rows(const int* counts, const uint32_t* remote_n, int cap, int* rows, GenMeta* gen,
                        hipStream_t stream);
// head of a window's graph: the next generation slot and the halo's per-age visibility cut-offs,
// tmax / ring state / other GPUs' row count reset, the window's row counts, and the fills of
// `fl` (see exchange.hip)
void launch_window_begin(const FillList& fl, GenMeta* gen, unsigned long long* tmax, int gens, long long halo_ns,
                         uint32_t* ring_state, uint32_t* remote_n, const int* counts, int cap, int* rows,
                         hipStream_t stream);

// join.hip
// rows [0, n_dev[0]) decoded by nblk blocks; with split (nblk_a < nblk) the first nblk_a blocks
// decoded rows [0, n_dev[0]) and the rest rows [n_dev[0], n_dev[1])
void launch_partition(const PartCodes* codes, const int* n_dev, int cap, int nblk, const uint32_t* part_blk,
                      uint32_t* part_off, uint32_t* part_tot, uint32_t* part_base, uint32_t* items,
                      hipStream_t stream, int nblk_a = 0);
// signals: the current generation's lists (gc.items / gc.keys / gc.base) from gc.part and gc.rec
// (bases_done: recorded after the partition bases, before the scatter -- the span branch's cue;
// work_*: the spans' list offsets, the join parameters and the probe's work list -- given, the
// scatter's launch also builds the work list (one extra workgroup), the spans' lists must exist)
struct JoinParams;
void launch_partition_sig(const SignalCols& gc, const int* n_dev, int cap, int nblk, const uint32_t* part_blk,
                          uint32_t* part_off, uint32_t* part_tot, hipStream_t stream, int nblk_a = 0,
                          hipEvent_t bases_done = nullptr, const uint32_t* work_span_base = nullptr,
                          const JoinParams* work_jp = nullptr, uint32_t* work = nullptr);
// A span at its position in a (key type, partition) list, the list sorted by (key hash, ts) in
// chunks of the probe's staging size: what the probe stages, written once per window
// (k_span_sort). run = the position's hash-run id in its chunk | run uniform << 16.
struct alignas(64) PreSpan {
  uint64_t h;
  int64_t t;
  uint64_t tr, cn;
  uint32_t pod, pid, sn, grp;
  uint32_t idx, run;
  uint32_t pad[2];
};
static_assert(sizeof(PreSpan) == 64, "one cache line per staged span");
// spans of this window x every visible generation's signals; span_pre: kKeyTypes * span_cap
// PreSpan of scratch
// (after launch_span_sort and launch_probe_work)
void launch_probe(const SpanCols& sc, const uint32_t* span_items, const uint32_t* span_base, const SignalCols& gc,
                  int span_cap, const JoinParams& jp, unsigned long long* top3, uint32_t* cnt, int n_groups,
                  unsigned long long* gsum, uint32_t* gcnt, unsigned long long* dbg, uint32_t* work,
                  PreSpan* span_pre, hipStream_t stream);
// every (key type, partition) span list sorted by (key hash, ts) into span_pre (k_span_sort)
void launch_span_sort(const SpanCols& sc, const uint32_t* span_items, const uint32_t* span_base, PreSpan* span_pre,
                      hipStream_t stream);
// the probe's work list from both sides' partition bases (k_probe_work, one workgroup)
void launch_probe_work(const uint32_t* span_base, const SignalCols& gc, const JoinParams& jp, uint32_t* work,
                       hipStream_t stream);
// probe work list: 4 header words + per phase one word per (key type, generation, partition,
// signal slice)
constexpr int kProbeMaxSplit = 64;  // signal slices per (key type, generation, partition); 8 bits of the item code
constexpr int kProbePhaseItems = kMaxGens * kParts * kProbeMaxSplit;  // per key type
// phase 1 (trace) holds one key type's items, phase 2 three
constexpr int kProbeProfOff = 4 + 4 * kProbePhaseItems;  // MISLO_PROBE_PROFILE counters (u64 [4][8])
constexpr int kProbeWorkLen = kProbeProfOff + 64;
void launch_finalize(const int* ns_dev, int span_cap, const unsigned long long* top3, const uint32_t* cnt,
                     const SignalCols& gc, const SpanCols& sc, const JoinParams& jp, const float* base_attrs,
                     float* attrs, float* conf, float* kernel_ms, int n_groups, unsigned long long* gsum, uint32_t* gcnt,
                     float* feat, unsigned long long* dbg, hipStream_t stream);

void launch_group_features(int n_groups, const unsigned long long* gsum, const uint32_t* gcnt, float* feat, hipStream_t stream);

// posterior.hip
// app / app_cnt (optional): the application evidence model and the groups' [G][2] retrieval counts
void launch_posterior(const float* feat, const int* ng_dev, int cap, const PosteriorModel* pm, const int32_t* labels,
                      double* post, int32_t* pred, double* conf, uint32_t* evbits, uint32_t* confusion,
                      hipStream_t stream, const AppModel* app = nullptr, const uint32_t* app_cnt = nullptr);
void launch_stats(const float* feat, const int* ng_dev, int cap, const PosteriorModel* pm, const int32_t* labels,
                  const float* weights, double* out, double* count, hipStream_t stream);

void launch_posterior_stats(const float* feat, const int* ng_dev, int cap, const PosteriorModel* pm,
                            const int32_t* labels, double* post, int32_t* pred, double* conf, uint32_t* evbits,
                            uint32_t* confusion, const int32_t* stat_labels, const float* weights, double* out,
                            double* count, hipStream_t stream, const AppModel* app = nullptr,
                            const uint32_t* app_cnt = nullptr);
void launch_refit_nb(double* stats, const double* add, const double* p0, double alpha, double prior_pseudo, int n_dom,
                     PosteriorModel* pm, hipStream_t stream, double inv_temp = 1.0, double min_count = 0.0,
                     const double* floor_tab = nullptr, int cap_dom = -1, double ceil = 1.0);

// gatestats.hip (K5)
int boot_max_n();
void launch_boot_quantile(const double* sorted_c, int nc, const double* sorted_b, int nb, double q, int iters,
                          uint64_t seed, double* out, hipStream_t stream);
void launch_rank_counts(const double* vals, int n_all, int nx, uint32_t* out, hipStream_t stream);

// storm.hip (K6)
void launch_storm_counts(const uint64_t* keys, const int64_t* ts, int n, int64_t window_ns, uint32_t threshold,
                         uint32_t* counts, unsigned long long* n_storm, hipStream_t stream);

}  // namespace mislo
