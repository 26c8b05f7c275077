// PyTorch bindings for the MI355X engine: a device-resident per-window Engine that owns
// every buffer (allocated once through the caching allocator, sized for the window
// capacity, so a window launches with no allocation and can be captured in a HIP graph)
// and drives decode -> partition -> LDS join -> finalize -> MFMA posterior -> stats on the
// caller's current HIP stream.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include <cmath>
#include <cstring>
#include <stdexcept>

#include "mislo_launch.h"
#include "mislo_packet_kernels.h"

namespace py = pybind11;
using namespace mislo;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define HIPCHECK(x)                                                                    \
  do {                                                                                 \
    hipError_t _e = (x);                                                               \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") +       \
                                                   hipGetErrorString(_e) + " at " #x); \
  } while (0)

template <typename T>
T* dptr(const torch::Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}

void check_cuda(const torch::Tensor& t, const char* name) {
  if (!t.is_cuda()) throw std::invalid_argument(std::string(name) + " must be a device tensor");
  if (!t.is_contiguous()) throw std::invalid_argument(std::string(name) + " must be contiguous");
}

}  // namespace

class Engine {
 public:
  Engine(int64_t sig_cap, int64_t span_cap, int64_t group_cap, int64_t device)
      : sig_cap_((int)sig_cap), span_cap_((int)span_cap), group_cap_((int)group_cap) {
    if (sig_cap <= 0 || span_cap <= 0 || group_cap <= 0) throw std::invalid_argument("capacities must be > 0");
    if (sig_cap >= (1LL << 27)) throw std::invalid_argument("sig_cap must be < 2^27 (top-3 key packing)");
    dev_ = torch::Device(torch::kCUDA, (c10::DeviceIndex)device);
    c10::hip::HIPGuard guard((c10::DeviceIndex)device);
    auto i64 = torch::TensorOptions().dtype(torch::kInt64).device(dev_);
    auto i32 = torch::TensorOptions().dtype(torch::kInt32).device(dev_);
    auto u8 = torch::TensorOptions().dtype(torch::kUInt8).device(dev_);
    auto f32 = torch::TensorOptions().dtype(torch::kFloat32).device(dev_);
    auto f64 = torch::TensorOptions().dtype(torch::kFloat64).device(dev_);
    const int64_t N = sig_cap_, S = span_cap_, G = group_cap_;
    nblk_sig_ = decode_grid(sig_cap_);
    nblk_span_ = decode_grid(span_cap_);
    counts = torch::zeros({kCountsLen}, i32);  // n_ev, n_spans, n_groups, n_local, base0 lo/hi, n_ctx, -, bases 1-3
    // signal columns
    // signals: 64-byte row records, status, partition codes of the 4 join keys
    g_status = torch::empty({N}, u8);
    g_part = torch::empty({N, 4}, torch::TensorOptions().dtype(torch::kInt16).device(dev_));
    g_part_blk = torch::empty({(int64_t)nblk_sig_ * kKeyTypes * kParts}, i32);
    g_part_off = torch::empty_like(g_part_blk);
    g_part_tot = torch::empty({kKeyTypes * kParts}, i32);
    g_part_base = torch::empty({kKeyTypes * kParts + 1}, i32);
    g_items = torch::empty({kKeyTypes * N}, i32);
    g_keys = torch::empty({kKeyTypes * N * (int64_t)sizeof(KeyTs)}, u8);
    g_rec = torch::empty({(int64_t)N * (int64_t)sizeof(SigRec)}, u8);
    // span columns
    s_part = torch::empty({S, 4}, torch::TensorOptions().dtype(torch::kInt16).device(dev_));
    s_part_blk = torch::empty({(int64_t)nblk_span_ * kKeyTypes * kParts}, i32);
    s_part_off = torch::empty_like(s_part_blk);
    s_part_tot = torch::empty({kKeyTypes * kParts}, i32);
    s_part_base = torch::empty({kKeyTypes * kParts + 1}, i32);
    s_items = torch::empty({kKeyTypes * S}, i32);
    s_pre = torch::empty({kKeyTypes * S * (int64_t)sizeof(PreSpan)}, u8);
    s_rec = torch::empty({(int64_t)S * (int64_t)sizeof(SpanRec)}, u8);
    probe_work = torch::zeros({kProbeWorkLen}, i32);
    top3 = torch::empty({3 * S}, i64); cnt = torch::empty({S}, i32);
    attrs = torch::empty({S, kSlots}, f32); conf = torch::empty({S}, f32); kernel_ms = torch::empty({S}, f32);
    // groups / incidents
    gsum = torch::empty({kGroupStripes * G, kSlots}, i64); gcnt = torch::empty({kGroupStripes * G, kSlots}, i32);
    feat = torch::empty({G, kSlots}, f32); labels = torch::full({G}, -1, i32);
    post = torch::empty({G, kMaxDomains}, f64); pred = torch::empty({G}, i32); gconf = torch::empty({G}, f64);
    evbits = torch::empty({G, kMaxDomains}, i32);
    // window accumulators
    hist = torch::empty({kSlots, kBuckets}, i32); status_cnt = torch::empty({kSlots, 3}, i32);
    misc = torch::empty({kPacketMisc}, i64); dbg = torch::empty({kPacketDbg}, i64);
    confusion = torch::empty({kMaxDomains, kMaxDomains}, i32);
    stats = torch::empty({32, 32}, f64); stats_count = torch::empty({kMaxDomains}, f64);
    packet = torch::empty({kPacketLen}, f64);
    ctx_table = torch::zeros({1, 4}, i32);
    model = torch::zeros({(int64_t)sizeof(PosteriorModel)}, u8);
    join_defaults();
  }

  void join_defaults() { set_join_params(2000.0, 0.7, 3, 1); }

  void set_join_params(double window_ms, double threshold, int64_t fanout, int64_t group_mode) {
    const int64_t ms = 1000000;
    int64_t outer = (int64_t)llround(window_ms * ms);
    if (outer <= 0) outer = 2000 * ms;
    if (outer >= (1LL << 35)) throw std::invalid_argument("window too large for top-3 key packing (< 34 s)");
    jp_.outer_ns = outer;
    const int64_t tw[4] = {outer, 100 * ms, 250 * ms, 500 * ms};
    for (int k = 0; k < 4; ++k) jp_.win_ns[k] = std::min(outer, tw[k]);
    const float cf[4] = {1.0f, 0.9f, 0.8f, 0.65f};
    for (int k = 0; k < 4; ++k) jp_.conf[k] = cf[k];
    jp_.threshold = threshold > 0 ? (float)threshold : 0.7f;
    if (fanout <= 0) fanout = 3;
    if (fanout > 3) throw std::invalid_argument("GPU join keeps at most 3 candidates per span");
    jp_.fanout = (int)fanout;
    jp_.group_mode = (int)group_mode;
  }

  // Retarget the per-window I/O buffers (counts int32[4], labels int32[group_cap],
  // packet f64[PACKET_LEN]) so the caller can double-buffer them: the H2D of window i+1
  // and the RCCL all-reduce of window i's packet then never race window i's kernels.
  void bind_io(torch::Tensor c, torch::Tensor l, torch::Tensor p) {
    check_cuda(c, "counts");
    check_cuda(l, "labels");
    check_cuda(p, "packet");
    if (c.scalar_type() != torch::kInt32 || c.numel() < 4) throw std::invalid_argument("counts: int32[4]");
    if (l.scalar_type() != torch::kInt32 || l.numel() < group_cap_) throw std::invalid_argument("labels: int32[G]");
    if (p.scalar_type() != torch::kFloat64 || p.numel() < kPacketLen) throw std::invalid_argument("packet: f64[L]");
    counts = c;
    labels = l;
    packet = p;
  }

  // Stream-ordered model update from a (pinned) host byte image of PosteriorModel.
  void set_model_bytes(torch::Tensor host_bytes) {
    if (host_bytes.scalar_type() != torch::kUInt8 || host_bytes.numel() != (int64_t)sizeof(PosteriorModel))
      throw std::invalid_argument("model image must be uint8[POSTERIOR_MODEL_BYTES]");
    model.copy_(host_bytes, /*non_blocking=*/true);
  }

  // ---- stages --------------------------------------------------------------------------
  void reset_window() {
    FillList fl{};
    auto add = [&](const torch::Tensor& t, uint32_t v) {
      fl.seg[fl.count++] = FillSeg{reinterpret_cast<uint32_t*>(t.data_ptr()), (uint32_t)(t.nbytes() / 4), v};
    };
    add(hist, 0); add(status_cnt, 0); add(misc, 0); add(dbg, 0); add(confusion, 0); add(stats, 0);
    add(stats_count, 0); add(top3, 0xFFFFFFFFu); add(cnt, 0); add(gsum, 0); add(gcnt, 0);
    hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, cur_stream(), fl);
  }

  // one generation (no halo): slot 0, every row local
  SignalCols sig_cols() {
    return SignalCols{reinterpret_cast<SigRec*>(g_rec.data_ptr()), dptr<uint8_t>(g_status),
                      reinterpret_cast<PartCodes*>(g_part.data_ptr()), dptr<uint32_t>(g_items),
                      reinterpret_cast<KeyTs*>(g_keys.data_ptr()), dptr<uint32_t>(g_part_base), nullptr,
                      (int64_t)sig_cap_, 1};
  }
  void partition_signals() {
    launch_partition_sig(sig_cols(), dptr<int>(counts), sig_cap_, nblk_sig_, dptr<uint32_t>(g_part_blk),
                         dptr<uint32_t>(g_part_off), dptr<uint32_t>(g_part_tot), cur_stream());
  }
  SpanCols span_cols() {
    return SpanCols{reinterpret_cast<SpanRec*>(s_rec.data_ptr()), reinterpret_cast<PartCodes*>(s_part.data_ptr())};
  }

  // events: device uint8 tensor of 64-byte records (>= n*64 bytes); counts[0] must hold n.
  void decode(torch::Tensor events) {
    check_cuda(events, "events");
    if (events.nbytes() < (size_t)sig_cap_ * 64)
      throw std::invalid_argument("events buffer must hold sig_cap 64-byte records");
    launch_decode_events(events.data_ptr(), dptr<int>(counts), sig_cap_, sig_cols(), dptr<uint32_t>(hist),
                         dptr<uint32_t>(status_cnt), dptr<uint32_t>(g_part_blk),
                         dptr<unsigned long long>(misc), cur_stream());
    partition_signals();
  }

  // context id -> {pod, pid, conn32, svc<<16|node} (int32 [n, 4]) for EVENT16 records and SPAN20 spans
  void set_ctx_table(torch::Tensor table) {
    check_cuda(table, "ctx_table");
    if (table.scalar_type() != torch::kInt32 || table.dim() != 2 || table.size(1) != 4 || !table.is_contiguous())
      throw std::invalid_argument("ctx_table must be contiguous int32 [n, 4]");
    ctx_table = table;
  }

  // events: device buffer of 16-byte EVENT16 records (>= sig_cap * 16 bytes); counts[4..5], [8..13] =
  // epoch bases, counts[6] = valid context-table rows (0 = all)
  void decode_ctx_wire(torch::Tensor events) {
    check_cuda(events, "events");
    if (events.nbytes() < (size_t)sig_cap_ * 16) throw std::invalid_argument("events buffer must hold sig_cap EVENT16 records");
    if (counts.numel() < 14) throw std::invalid_argument("EVENT16 windows need counts int32[>= 14] (epoch bases)");
    launch_decode_wire(events.data_ptr(), dptr<int>(counts), sig_cap_, dptr<uint32_t>(ctx_table),
                       (int)ctx_table.size(0), sig_cols(), dptr<uint32_t>(hist), dptr<uint32_t>(status_cnt),
                       dptr<uint32_t>(g_part_blk), dptr<unsigned long long>(misc), cur_stream());
    partition_signals();
  }

  void decode_wire(torch::Tensor events, int64_t wire) {
    if (wire == 16) decode_ctx_wire(events);
    else if (wire == 64) decode(events);
    else throw std::invalid_argument("wire must be 64 (EVENT) or 16 (EVENT16)");
  }

  void decode_ref(torch::Tensor events, int64_t pod, int64_t svcnode, int64_t trace_h) {
    check_cuda(events, "events");
    if (events.nbytes() < (size_t)sig_cap_ * 40)
      throw std::invalid_argument("events buffer must hold sig_cap 40-byte REF records");
    launch_decode_ref(events.data_ptr(), dptr<int>(counts), sig_cap_, (uint32_t)pod, (uint32_t)svcnode,
                      (uint64_t)trace_h, sig_cols(), dptr<uint32_t>(hist), dptr<uint32_t>(status_cnt),
                      dptr<uint32_t>(g_part_blk), dptr<unsigned long long>(misc), cur_stream());
    partition_signals();
  }

  // spans: device uint8 tensor of 64-byte span records; counts[1] = n spans, counts[2] = n groups
  void join(torch::Tensor spans, int64_t n_groups, c10::optional<torch::Tensor> base_attrs) {
    check_cuda(spans, "spans");
    if (spans.nbytes() < (size_t)span_cap_ * 64)
      throw std::invalid_argument("spans buffer must hold span_cap 64-byte records");
    if (n_groups > group_cap_) throw std::invalid_argument("n_groups exceeds group capacity");
    hipStream_t st = cur_stream();
    if (counts.numel() < 8) throw std::invalid_argument("counts must hold int32[>= 8] (counts[7] = span record bytes)");
    launch_decode_spans(spans.data_ptr(), dptr<int>(counts) + 1, span_cap_, span_cols(), dptr<uint32_t>(s_part_blk),
                        dptr<uint32_t>(ctx_table), (int)ctx_table.size(0), st);
    launch_partition(reinterpret_cast<const PartCodes*>(s_part.data_ptr()), dptr<int>(counts) + 1, span_cap_, nblk_span_,
                     dptr<uint32_t>(s_part_blk), dptr<uint32_t>(s_part_off), dptr<uint32_t>(s_part_tot),
                     dptr<uint32_t>(s_part_base), dptr<uint32_t>(s_items), st);
    // top3 / cnt / gsum / gcnt were reset by reset_window()
    launch_span_sort(span_cols(), dptr<uint32_t>(s_items), dptr<uint32_t>(s_part_base),
                     reinterpret_cast<PreSpan*>(s_pre.data_ptr()), st);
    launch_probe_work(dptr<uint32_t>(s_part_base), sig_cols(), jp_, dptr<uint32_t>(probe_work), st);
    launch_probe(span_cols(), dptr<uint32_t>(s_items), dptr<uint32_t>(s_part_base), sig_cols(), span_cap_, jp_,
                 dptr<unsigned long long>(top3), dptr<uint32_t>(cnt), (int)n_groups, dptr<unsigned long long>(gsum),
                 dptr<uint32_t>(gcnt), dptr<unsigned long long>(dbg), dptr<uint32_t>(probe_work),
                 reinterpret_cast<PreSpan*>(s_pre.data_ptr()), st);
    const float* base = nullptr;
    if (base_attrs.has_value()) {
      check_cuda(*base_attrs, "base_attrs");
      if (base_attrs->numel() < (int64_t)span_cap_ * kSlots || base_attrs->scalar_type() != torch::kFloat32)
        throw std::invalid_argument("base_attrs must be float32 [span_cap, 16]");
      base = base_attrs->data_ptr<float>();
    }
    launch_finalize(dptr<int>(counts) + 1, span_cap_, dptr<unsigned long long>(top3), dptr<uint32_t>(cnt), sig_cols(),
                    span_cols(), jp_, base, dptr<float>(attrs), dptr<float>(conf), dptr<float>(kernel_ms),
                    (int)n_groups, dptr<unsigned long long>(gsum), dptr<uint32_t>(gcnt), dptr<float>(feat),
                    dptr<unsigned long long>(dbg), st);
  }

  // Incident features -> posteriors (counts[2] = number of incident rows in `feat`).
  void posterior(bool with_labels) {
    launch_posterior(dptr<float>(feat), dptr<int>(counts) + 2, group_cap_,
                     reinterpret_cast<const PosteriorModel*>(model.data_ptr()),
                     with_labels ? dptr<int32_t>(labels) : nullptr, dptr<double>(post), dptr<int32_t>(pred),
                     dptr<double>(gconf), dptr<uint32_t>(evbits), dptr<uint32_t>(confusion), cur_stream());
  }

  void accumulate_stats(c10::optional<torch::Tensor> weights) {
    const float* w = nullptr;
    if (weights.has_value()) {
      check_cuda(*weights, "weights");
      w = weights->data_ptr<float>();
    }
    launch_stats(dptr<float>(feat), dptr<int>(counts) + 2, group_cap_,
                 reinterpret_cast<const PosteriorModel*>(model.data_ptr()), dptr<int32_t>(labels), w,
                 dptr<double>(stats), dptr<double>(stats_count), cur_stream());
  }

  // posterior(with_labels) + accumulate_stats() of a learning window as one launch
  void posterior_and_stats(bool with_labels) {
    launch_posterior_stats(dptr<float>(feat), dptr<int>(counts) + 2, group_cap_,
                           reinterpret_cast<const PosteriorModel*>(model.data_ptr()),
                           with_labels ? dptr<int32_t>(labels) : nullptr, dptr<double>(post), dptr<int32_t>(pred),
                           dptr<double>(gconf), dptr<uint32_t>(evbits), dptr<uint32_t>(confusion),
                           dptr<int32_t>(labels), nullptr, dptr<double>(stats), dptr<double>(stats_count),
                           cur_stream());
  }

  void pack() {
    hipLaunchKernelGGL(k_pack, dim3((kPacketLen + 255) / 256), dim3(256), 0, cur_stream(), dptr<uint32_t>(hist),
                       dptr<uint32_t>(status_cnt), dptr<unsigned long long>(misc), dptr<unsigned long long>(dbg),
                       dptr<uint32_t>(confusion), dptr<double>(stats), dptr<double>(stats_count), nullptr,
                       dptr<double>(packet));
  }

  // Full window: expects events/spans already resident and counts = [n_ev, n_spans, n_groups, 0, ...].
  // wire: 64 = Event records, 16 = EVENT16
  void run_window(torch::Tensor events, torch::Tensor spans, int64_t n_groups, bool with_labels, bool learn,
                  int64_t wire) {
    reset_window();
    decode_wire(events, wire);
    join(spans, n_groups, c10::nullopt);
    if (learn) posterior_and_stats(with_labels);
    else posterior(with_labels);
    pack();
  }

  // Global incident scope, split at the group-sum all-reduce (parallel/__init__.py):
  //   run_window_pre -> all_reduce(gsum), all_reduce(gcnt) -> run_window_post
  void run_window_pre(torch::Tensor events, torch::Tensor spans, int64_t n_groups, int64_t wire) {
    reset_window();
    decode_wire(events, wire);
    join(spans, n_groups, c10::nullopt);
  }

  void run_window_post(int64_t n_groups, bool with_labels, bool learn) {
    if (n_groups > group_cap_) throw std::invalid_argument("n_groups exceeds group capacity");
    launch_group_features((int)n_groups, dptr<unsigned long long>(gsum), dptr<uint32_t>(gcnt), dptr<float>(feat), cur_stream());
    if (learn) posterior_and_stats(with_labels);
    else posterior(with_labels);
    pack();
  }

  // On-device learned-NB refit from accumulated stats ([32*32 + 16] f64) and the Beta prior's
  // table p0 ([16*16] f64, optionally followed by a [16*16] likelihood floor); rewrites the model
  // in place (stream order). add (optional, f64[1040]): statistics folded into stats_acc first,
  // in the same launch. cap_dom >= 0: that domain's prior capped at the others' largest.
  void refit_nb(torch::Tensor stats_acc, torch::Tensor p0, double alpha, double prior_pseudo, int64_t n_dom,
                c10::optional<torch::Tensor> add, int64_t cap_dom) {
    check_cuda(stats_acc, "stats_acc");
    check_cuda(p0, "p0");
    if (stats_acc.scalar_type() != torch::kFloat64 || stats_acc.numel() < 32 * 32 + kMaxDomains ||
        !stats_acc.is_contiguous())
      throw std::invalid_argument("stats_acc must be contiguous f64[1040]");
    if (p0.scalar_type() != torch::kFloat64 || p0.numel() < kSlots * 16) throw std::invalid_argument("p0: f64[256]");
    if (n_dom < 1 || n_dom > kMaxDomains) throw std::invalid_argument("n_dom out of range");
    const double* addp = nullptr;
    if (add && add->defined()) {
      check_cuda(*add, "add");
      if (add->scalar_type() != torch::kFloat64 || add->numel() < 32 * 32 + kMaxDomains || !add->is_contiguous())
        throw std::invalid_argument("add must be contiguous f64[1040]");
      addp = add->data_ptr<double>();
    }
    if (cap_dom >= n_dom) throw std::invalid_argument("cap_dom out of range");
    const double* floor_tab = p0.numel() >= 2 * kSlots * 16 ? p0.data_ptr<double>() + kSlots * 16 : nullptr;
    launch_refit_nb(stats_acc.data_ptr<double>(), addp, p0.data_ptr<double>(), alpha, prior_pseudo, (int)n_dom,
                    reinterpret_cast<PosteriorModel*>(model.data_ptr()), cur_stream(), 1.0, 0.0, floor_tab,
                    (int)cap_dom);
  }

  int64_t sig_cap() const { return sig_cap_; }
  int64_t span_cap() const { return span_cap_; }
  int64_t group_cap() const { return group_cap_; }
  int64_t packet_len() const { return kPacketLen; }

  torch::Tensor counts;
  torch::Tensor g_status, g_part;
  torch::Tensor g_part_blk, g_part_off, g_part_tot, g_part_base, g_items, g_keys, g_rec, s_rec;
  torch::Tensor s_part;
  torch::Tensor s_part_blk, s_part_off, s_part_tot, s_part_base, s_items, s_pre, probe_work;
  torch::Tensor top3, cnt, attrs, conf, kernel_ms;
  torch::Tensor gsum, gcnt, feat, labels, post, pred, gconf, evbits;
  torch::Tensor hist, status_cnt, misc, dbg, confusion, stats, stats_count, packet, model, ctx_table;

 private:
  int sig_cap_, span_cap_, group_cap_;
  int nblk_sig_ = 1, nblk_span_ = 1;
  torch::Device dev_{torch::kCPU};
  JoinParams jp_{};
};

void set_tables_py(torch::Tensor type_slot, torch::Tensor scale, torch::Tensor warn, torch::Tensor err,
                   torch::Tensor edges) {
  Tables t;
  std::memset(&t, 0, sizeof(t));
  auto ts = type_slot.to(torch::kCPU, torch::kInt8).contiguous();
  auto sc = scale.to(torch::kCPU, torch::kFloat32).contiguous();
  auto wa = warn.to(torch::kCPU, torch::kFloat32).contiguous();
  auto er = err.to(torch::kCPU, torch::kFloat32).contiguous();
  auto ed = edges.to(torch::kCPU, torch::kFloat32).contiguous();
  if (ts.numel() != kMaxTypes || sc.numel() != kSlots || ed.numel() != kSlots * kBuckets)
    throw std::invalid_argument("table shapes");
  std::memcpy(t.type_slot, ts.data_ptr<int8_t>(), sizeof(t.type_slot));
  std::memcpy(t.scale, sc.data_ptr<float>(), sizeof(t.scale));
  std::memcpy(t.warn, wa.data_ptr<float>(), sizeof(t.warn));
  std::memcpy(t.err, er.data_ptr<float>(), sizeof(t.err));
  std::memcpy(t.edges, ed.data_ptr<float>(), sizeof(t.edges));
  set_tables(&t);
}

// ---- K5 gate statistics / K6 storm counts (stand-alone device ops) -----------------------
static void check_dev(const torch::Tensor& t, torch::ScalarType st, const char* name) {
  check_cuda(t, name);
  if (t.scalar_type() != st) throw std::invalid_argument(std::string(name) + ": wrong dtype");
}

// sorted_c / sorted_b: ascending f64 samples; returns [2, iters] bootstrap quantiles
torch::Tensor boot_quantile_py(torch::Tensor sorted_c, torch::Tensor sorted_b, double q, int64_t iters,
                               int64_t seed) {
  check_dev(sorted_c, torch::kFloat64, "sorted_c");
  check_dev(sorted_b, torch::kFloat64, "sorted_b");
  const int64_t nc = sorted_c.numel(), nb = sorted_b.numel();
  if (nc < 1 || nb < 1 || nc > boot_max_n() || nb > boot_max_n())
    throw std::invalid_argument("bootstrap sample sizes must be in [1, boot_max_n]");
  if (iters < 1 || iters >= (1LL << 31)) throw std::invalid_argument("iters out of range");
  if (!(q >= 0.0 && q <= 1.0)) throw std::invalid_argument("q must be in [0, 1]");
  c10::hip::HIPGuard guard(sorted_c.device().index());
  auto out = torch::empty({2, iters}, sorted_c.options());
  launch_boot_quantile(sorted_c.data_ptr<double>(), (int)nc, sorted_b.data_ptr<double>(), (int)nb, q, (int)iters,
                       (uint64_t)seed, out.data_ptr<double>(), cur_stream());
  return out;
}

// vals: [x..., y...] f64; returns uint32-as-int32 [4, n]: (all<v, all==v, y<v, y>v)
torch::Tensor rank_counts_py(torch::Tensor vals, int64_t nx) {
  check_dev(vals, torch::kFloat64, "vals");
  const int64_t n = vals.numel();
  if (nx < 0 || nx > n || n >= (1LL << 31)) throw std::invalid_argument("nx out of range");
  c10::hip::HIPGuard guard(vals.device().index());
  auto out = torch::empty({4, n}, vals.options().dtype(torch::kInt32));
  if (n) launch_rank_counts(vals.data_ptr<double>(), (int)n, (int)nx, dptr<uint32_t>(out), cur_stream());
  return out;
}

// keys (int64, sorted), ts (int64, sorted within key): per-event window counts + storm tally
std::tuple<torch::Tensor, torch::Tensor> storm_counts_py(torch::Tensor keys, torch::Tensor ts, int64_t window_ns,
                                                         int64_t threshold) {
  check_dev(keys, torch::kInt64, "keys");
  check_dev(ts, torch::kInt64, "ts");
  const int64_t n = keys.numel();
  if (ts.numel() != n || n >= (1LL << 31)) throw std::invalid_argument("keys/ts size mismatch");
  c10::hip::HIPGuard guard(keys.device().index());
  auto counts = torch::empty({n}, keys.options().dtype(torch::kInt32));
  auto tally = torch::zeros({1}, keys.options());
  launch_storm_counts(dptr<uint64_t>(keys), ts.data_ptr<int64_t>(), (int)n, window_ns, (uint32_t)threshold,
                      dptr<uint32_t>(counts), dptr<unsigned long long>(tally), cur_stream());
  return {counts, tally};
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X (gfx950) LLM-SLO engine kernels";
  m.def("set_tables", &set_tables_py);
  m.def("boot_quantile", &boot_quantile_py, py::arg("sorted_c"), py::arg("sorted_b"), py::arg("q"),
        py::arg("iters"), py::arg("seed"));
  m.def("rank_counts", &rank_counts_py, py::arg("vals"), py::arg("nx"));
  m.def("storm_counts", &storm_counts_py, py::arg("keys"), py::arg("ts"), py::arg("window_ns"),
        py::arg("threshold"));
  m.attr("BOOT_MAX_N") = boot_max_n();
  m.attr("PACKET_LEN") = kPacketLen;
  m.attr("PACKET_LAYOUT") = py::make_tuple(kPacketHist, kPacketStatus, kPacketMisc, kPacketDbg, kPacketConf,
                                           kPacketStats, kPacketCount);
  m.attr("PARTS") = kParts;
  m.attr("POSTERIOR_MODEL_BYTES") = (int64_t)sizeof(PosteriorModel);
  m.attr("PROBE_PROF_OFF") = kProbeProfOff;
  py::class_<Engine>(m, "Engine")
      .def(py::init<int64_t, int64_t, int64_t, int64_t>(), py::arg("sig_cap"), py::arg("span_cap"),
           py::arg("group_cap"), py::arg("device") = 0)
      .def("set_join_params", &Engine::set_join_params, py::arg("window_ms") = 2000.0,
           py::arg("threshold") = 0.7, py::arg("fanout") = 3, py::arg("group_mode") = 1)
      .def("set_model_bytes", &Engine::set_model_bytes)
      .def("bind_io", &Engine::bind_io)
      .def("reset_window", &Engine::reset_window)
      .def("decode", &Engine::decode)
      .def("decode_ref", &Engine::decode_ref)
      .def("set_ctx_table", &Engine::set_ctx_table)
      .def("decode_ctx_wire", &Engine::decode_ctx_wire)
      .def("decode_wire", &Engine::decode_wire)
      .def("join", &Engine::join, py::arg("spans"), py::arg("n_groups"), py::arg("base_attrs") = py::none())
      .def("posterior", &Engine::posterior)
      .def("accumulate_stats", &Engine::accumulate_stats, py::arg("weights") = py::none())
      .def("pack", &Engine::pack)
      .def("run_window", &Engine::run_window, py::arg("events"), py::arg("spans"), py::arg("n_groups"),
           py::arg("with_labels") = true, py::arg("learn") = false, py::arg("wire") = 64)
      .def("refit_nb", &Engine::refit_nb, py::arg("stats_acc"), py::arg("p0"), py::arg("alpha") = 2.0,
           py::arg("prior_pseudo") = 1.0, py::arg("n_dom") = 10, py::arg("add") = py::none(), py::arg("cap_dom") = -1)
      .def("run_window_pre", &Engine::run_window_pre, py::arg("events"), py::arg("spans"), py::arg("n_groups"),
           py::arg("wire") = 64)
      .def("run_window_post", &Engine::run_window_post, py::arg("n_groups"), py::arg("with_labels") = true,
           py::arg("learn") = false)
      .def_property_readonly("sig_cap", &Engine::sig_cap)
      .def_property_readonly("span_cap", &Engine::span_cap)
      .def_property_readonly("group_cap", &Engine::group_cap)
      .def_property_readonly("packet_len", &Engine::packet_len)
#define RO(name) .def_readonly(#name, &Engine::name)
      RO(counts) RO(g_rec) RO(g_status) RO(g_part) RO(g_part_base) RO(g_items) RO(s_rec) RO(s_part)
      RO(s_part_base) RO(s_items) RO(probe_work)
      RO(top3) RO(cnt) RO(attrs) RO(conf) RO(kernel_ms) RO(gsum) RO(gcnt) RO(feat) RO(labels) RO(post)
      RO(pred) RO(gconf) RO(evbits) RO(hist) RO(status_cnt) RO(misc) RO(dbg) RO(confusion) RO(stats)
      RO(stats_count) RO(packet) RO(model) RO(ctx_table);
#undef RO
}
