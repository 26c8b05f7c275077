// pybind11 module `_mislo_agent`: the native window engine (engine.h) for the agent daemon and
// the benchmark. No PyTorch: the agent process links the HIP runtime, RCCL and these kernels
// only (its resident set is part of the overhead budget, REF docs/benchmarks targets <= 250 MB).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>
#include <stdexcept>

#include "engine.h"

namespace py = pybind11;
using namespace mislo;

namespace {

template <class T>
py::array_t<T> copy_array(const T* p, std::vector<py::ssize_t> shape) {
  py::array_t<T> a(shape);
  size_t n = 1;
  for (auto s : shape) n *= (size_t)s;
  if (n) std::memcpy(a.mutable_data(), p, n * sizeof(T));
  return a;
}

void set_tables_np(py::array_t<int8_t, py::array::c_style | py::array::forcecast> type_slot,
                   py::array_t<float, py::array::c_style | py::array::forcecast> scale,
                   py::array_t<float, py::array::c_style | py::array::forcecast> warn,
                   py::array_t<float, py::array::c_style | py::array::forcecast> err,
                   py::array_t<float, py::array::c_style | py::array::forcecast> edges) {
  Tables t;
  std::memset(&t, 0, sizeof(t));
  if (type_slot.size() != kMaxTypes || scale.size() != kSlots || warn.size() != kSlots || err.size() != kSlots ||
      edges.size() != kSlots * kBuckets)
    throw std::invalid_argument("table shapes");
  std::memcpy(t.type_slot, type_slot.data(), sizeof(t.type_slot));
  std::memcpy(t.scale, scale.data(), sizeof(t.scale));
  std::memcpy(t.warn, warn.data(), sizeof(t.warn));
  std::memcpy(t.err, err.data(), sizeof(t.err));
  std::memcpy(t.edges, edges.data(), sizeof(t.edges));
  engine_set_tables(t);
}

}  // namespace

class PyEngine {
 public:
  PyEngine(int device, int sig_cap, int span_cap, int group_cap, int user_cap, int n_buffers, int max_ahead,
           double window_ms, double threshold, int fanout, int group_mode, bool use_graphs, bool device_refit,
           int n_dom, float ttft_slo_ms, double halo_ms, int import_cap, int xchg_cap, int shard_rank,
           int shard_world, int halo_windows, bool split_rings) {
    if (shard_world < 1 || shard_rank < 0 || shard_rank >= shard_world) throw std::invalid_argument("shard rank / world");
    EngineConfig c;
    c.device = device;
    c.sig_cap = sig_cap;
    c.span_cap = span_cap;
    c.group_cap = group_cap;
    c.user_cap = user_cap;
    c.n_buffers = n_buffers;
    c.max_ahead = max_ahead;
    c.window_ms = window_ms;
    c.threshold = threshold;
    c.fanout = fanout;
    c.group_mode = group_mode;
    c.use_graphs = use_graphs;
    c.device_refit = device_refit;
    c.n_dom = n_dom;
    c.ttft_slo_ms = ttft_slo_ms;
    c.halo_ms = halo_ms;
    c.halo_windows = halo_windows;
    c.import_cap = import_cap;
    c.xchg_cap = xchg_cap;
    c.shard_rank = shard_rank;
    c.shard_world = shard_world;
    c.split_rings = split_rings;
    e_ = std::make_unique<WindowEngine>(c);
  }
  bool register_host(uintptr_t addr, size_t bytes) {
    return e_->register_host(reinterpret_cast<const void*>(addr), bytes);
  }
  // segments: lists of (host address, bytes) in ring order
  void submit(int64_t k, const std::vector<std::pair<uintptr_t, size_t>>& kernel,
              const std::vector<std::pair<uintptr_t, size_t>>& user,
              const std::vector<std::pair<uintptr_t, size_t>>& spans, int n_groups, py::object labels,
              std::vector<int64_t> bases, bool with_labels, bool learn, int user_rec) {
    WindowInput in;
    auto conv = [](const std::vector<std::pair<uintptr_t, size_t>>& v, std::vector<Seg>& out) {
      for (auto& p : v) out.push_back(Seg{reinterpret_cast<const void*>(p.first), p.second});
    };
    conv(kernel, in.kernel);
    conv(user, in.user);
    conv(spans, in.spans);
    in.n_groups = n_groups;
    in.user_rec = user_rec;
    std::vector<int32_t> lab;
    if (!labels.is_none()) {
      auto arr = labels.cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
      lab.assign(arr.data(), arr.data() + arr.size());
      lab.resize(std::max<size_t>(lab.size(), (size_t)std::max(0, n_groups)), -1);
      in.labels = lab.data();
    }
    bases.resize(4, 0);
    for (int q = 0; q < 4; ++q) in.bases[q] = bases[q];
    py::gil_scoped_release nogil;
    e_->submit(k, in, with_labels, learn);
  }
  bool h2d_done(int64_t k) { return e_->h2d_done(k); }
  void wait_h2d(int64_t k) {
    py::gil_scoped_release nogil;
    e_->wait_h2d(k);
  }
  bool query(int64_t k) { return e_->query(k); }
  void wait(int64_t k) {
    py::gil_scoped_release nogil;
    e_->wait(k);
  }
  py::array_t<double> packet(int64_t k) { return copy_array(e_->packet(k), {kPacketLen}); }
  py::dict results(int64_t k, int n_groups) {
    if (n_groups < 0 || n_groups > eng().config().group_cap) throw std::invalid_argument("n_groups");
    return result_dict(e_->results(k), n_groups);
  }
  // every rank's results of window k (the node-wide incident list, all-gathered over RCCL)
  py::list results_all(int64_t k, int n_groups) {
    WindowEngine& e = eng();
    if (n_groups < 0 || n_groups > e.config().group_cap) throw std::invalid_argument("n_groups");
    const size_t G = e.config().group_cap, bytes = e.result_bytes();
    const uint8_t* base = e.results_all(k);
    const size_t o_gconf = 16 * G * 8, o_feat = o_gconf + G * 8, o_pred = o_feat + 16 * G * 4, o_ev = o_pred + G * 4;
    const size_t o_sli = o_ev + 16 * G * 4;
    py::list out;
    const int w = e.has_comm() ? e.world() : 1;
    for (int r = 0; r < w; ++r) {
      const uint8_t* p = base + (size_t)r * bytes;
      out.append(result_dict(ResultView{reinterpret_cast<const double*>(p), reinterpret_cast<const double*>(p + o_gconf),
                                        reinterpret_cast<const float*>(p + o_feat),
                                        reinterpret_cast<const int32_t*>(p + o_pred),
                                        reinterpret_cast<const uint32_t*>(p + o_ev),
                                        reinterpret_cast<const uint32_t*>(p + o_sli),
                                        reinterpret_cast<const uint32_t*>(p + o_sli) + 2 * G,
                                        reinterpret_cast<const uint32_t*>(p + o_sli) + 4 * G},
                             n_groups));
    }
    return out;
  }
  static py::dict result_dict(const ResultView& r, int n_groups) {
    const py::ssize_t G = n_groups;
    py::dict d;
    d["post"] = copy_array(r.post, {G, 16});
    d["conf"] = copy_array(r.gconf, {G});
    d["feat"] = copy_array(r.feat, {G, 16});
    d["pred"] = copy_array(r.pred, {G});
    d["evbits"] = copy_array(r.evbits, {G, 16});
    d["sli"] = copy_array(r.sli, {G, 2});
    d["app"] = copy_array(r.app, {G, 2});
    d["late"] = copy_array(r.late, {G, 2});
    return d;
  }
  py::tuple window_ms(int64_t k) {
    std::pair<float, float> t;
    {
      py::gil_scoped_release nogil;
      t = e_->window_ms(k);
    }
    return py::make_tuple(t.first, t.second);
  }
  void set_model_bytes(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> b) {
    e_->set_model_bytes(b.data(), (size_t)b.size());
  }
  void set_app_model(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> b) {
    e_->set_app_model(b.data(), (size_t)b.size());
  }
  void set_refit(double alpha, double prior_pseudo, double inv_temp, double min_count, int cap_dom, double ceil) {
    eng().set_refit(alpha, prior_pseudo, inv_temp, min_count, cap_dom, ceil);
  }
  void refit_now() { eng().refit_now(); }
  // K3 on given features (REF's 55 rows, offline evaluation) with the model on the device
  py::dict score(py::array_t<float, py::array::c_style | py::array::forcecast> feat, py::object labels,
                 py::object app) {
    if (feat.ndim() != 2 || feat.shape(1) != 16) throw std::invalid_argument("feat must be float32 [n, 16]");
    const int n = (int)feat.shape(0);
    std::vector<int32_t> lab;
    if (!labels.is_none()) {
      auto a = labels.cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
      if (a.size() != n) throw std::invalid_argument("labels must have n entries");
      lab.assign(a.data(), a.data() + n);
    }
    std::vector<uint32_t> appc;
    if (!app.is_none()) {
      auto a = app.cast<py::array_t<uint32_t, py::array::c_style | py::array::forcecast>>();
      if (a.size() != 2 * (py::ssize_t)n) throw std::invalid_argument("app must be uint32 [n, 2]");
      appc.assign(a.data(), a.data() + 2 * (size_t)n);
    }
    std::vector<double> post((size_t)n * 16), conf(n);
    std::vector<int32_t> pred(n);
    std::vector<uint32_t> ev((size_t)n * 16), cm(256);
    {
      py::gil_scoped_release nogil;
      eng().score_features(feat.data(), n, lab.empty() ? nullptr : lab.data(), post.data(), pred.data(), conf.data(),
                           ev.data(), cm.data(), appc.empty() ? nullptr : appc.data());
    }
    py::dict d;
    d["post"] = copy_array(post.data(), {n, 16});
    d["pred"] = copy_array(pred.data(), {n});
    d["conf"] = copy_array(conf.data(), {n});
    d["evbits"] = copy_array(ev.data(), {n, 16});
    d["confusion"] = copy_array(cm.data(), {16, 16});
    return d;
  }
  void set_p0(py::array_t<double, py::array::c_style | py::array::forcecast> p0) {
    if (p0.size() != kSlots * 16 && p0.size() != 2 * kSlots * 16)
      throw std::invalid_argument("p0 must be f64[256] (table) or f64[512] (table, floor)");
    e_->set_p0(p0.data(), (size_t)p0.size());
  }
  void set_pods(py::array_t<uint32_t, py::array::c_style | py::array::forcecast> pods,
                py::array_t<uint32_t, py::array::c_style | py::array::forcecast> sn) {
    if (pods.size() != sn.size()) throw std::invalid_argument("pods / svcnode size mismatch");
    e_->set_pods(pods.data(), sn.data(), (size_t)pods.size());
  }
  void inject_remote(py::buffer blocks, size_t stride, int world, int me) {
    py::buffer_info bi = blocks.request();
    if ((size_t)(bi.size * bi.itemsize) < stride * (size_t)std::max(world, 0)) throw std::invalid_argument("blocks too small");
    py::gil_scoped_release nogil;
    eng().inject_remote(bi.ptr, stride, world, me);
  }
  void set_join_params(double window_ms, double threshold, int fanout, int group_mode) {
    e_->set_join_params(window_ms, threshold, fanout, group_mode);
  }
  void init_comm(py::bytes id, int rank, int world) {
    std::string s = id;
    if (s.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("unique id size");
    ncclUniqueId u;
    std::memcpy(&u, s.data(), sizeof(u));
    py::gil_scoped_release nogil;
    e_->init_comm(u, rank, world);
  }
  py::array_t<double> totals() {
    std::vector<double> t(kPacketLen);
    {
      py::gil_scoped_release nogil;
      e_->totals(t.data());
    }
    return copy_array(t.data(), {kPacketLen});
  }
  void reset_totals() {
    py::gil_scoped_release nogil;
    e_->reset_totals();
  }
  py::array_t<double> stats_acc() {
    std::vector<double> t(kStatsLen);
    {
      py::gil_scoped_release nogil;
      e_->stats_acc(t.data());
    }
    return copy_array(t.data(), {kStatsLen});
  }
  void restore(py::array_t<double, py::array::c_style | py::array::forcecast> stats,
               py::array_t<uint8_t, py::array::c_style | py::array::forcecast> model, int64_t folded) {
    if (stats.size() != kStatsLen) throw std::invalid_argument("stats must be f64[STATS_LEN]");
    eng().restore(stats.data(), model.data(), (size_t)model.size(), folded);
  }
  py::array_t<uint8_t> model_bytes() {
    std::vector<uint8_t> t(sizeof(PosteriorModel));
    {
      py::gil_scoped_release nogil;
      e_->model_bytes(t.data());
    }
    return copy_array(t.data(), {(py::ssize_t)t.size()});
  }
  void sync() {
    py::gil_scoped_release nogil;
    e_->sync();
  }
  std::vector<int64_t> import_state() {
    py::gil_scoped_release nogil;
    return eng().import_state();
  }
  py::bytes sent_block() {
    std::vector<uint8_t> b;
    {
      py::gil_scoped_release nogil;
      b = eng().sent_block();
    }
    return py::bytes(reinterpret_cast<const char*>(b.data()), b.size());
  }
  void close() {
    if (e_) {
      py::gil_scoped_release nogil;
      e_->sync();
      e_.reset();
    }
  }
  WindowEngine& eng() {
    if (!e_) throw std::logic_error("engine closed");
    return *e_;
  }
  int buffers() { return eng().buffers(); }
  int64_t folded() { return eng().windows_folded(); }
  size_t graphs() { return eng().graphs(); }
  double host_issue_us() { return eng().host_issue_us(); }
  double host_wait_us() { return eng().host_wait_us(); }
  double host_dma_issue_us() { return eng().host_dma_issue_us(); }
  double host_launch_us() { return eng().host_launch_us(); }
  bool has_comm() { return eng().has_comm(); }
  size_t staged_bytes() { return eng().staged_bytes(); }
  size_t direct_bytes() { return eng().direct_bytes(); }

 private:
  std::unique_ptr<WindowEngine> e_;
};

py::bytes unique_id() {
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) throw std::runtime_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  return py::bytes(reinterpret_cast<const char*>(&u), sizeof(u));
}

PYBIND11_MODULE(_mislo_agent, m) {
  m.doc() = "MI355X LLM-SLO native window engine (HIP + RCCL, no PyTorch)";
  m.def("set_tables", &set_tables_np);
  m.def("unique_id", &unique_id);
  m.def("device_count", []() {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
  });
  m.attr("PACKET_LEN") = kPacketLen;
  m.attr("PACKET_LAYOUT") = py::make_tuple(kPacketHist, kPacketStatus, kPacketMisc, kPacketDbg, kPacketConf,
                                           kPacketStats, kPacketCount, kPacketRing);
  m.attr("STATS_OFF") = kStatsOff;
  m.attr("STATS_LEN") = kStatsLen;
  m.attr("POSTERIOR_MODEL_BYTES") = (int64_t)sizeof(PosteriorModel);
  m.attr("APP_MODEL_BYTES") = (int64_t)sizeof(AppModel);
  m.attr("APP_EVIDENCE_BIT") = kAppBit;
  m.attr("CTX_ROWS") = kCtxRows;
  m.attr("REC_STRIDE") = kRecStride;
  m.attr("SIGREC_BYTES") = (int)sizeof(SigRec);
  m.attr("RING_STATE") =
      py::make_tuple("first_busy", "foreign", "def_ctx", "def_trace", "discarded", "events", "other_shard");
  py::class_<PyEngine>(m, "WindowEngine")
      .def(py::init<int, int, int, int, int, int, int, double, double, int, int, bool, bool, int, float, double, int,
                    int, int, int, int, bool>(),
           py::arg("device") = 0, py::arg("sig_cap") = 1 << 20, py::arg("span_cap") = 16384, py::arg("group_cap") = 64,
           py::arg("user_cap") = 1 << 18, py::arg("n_buffers") = 3, py::arg("max_ahead") = 3,
           py::arg("window_ms") = 2000.0, py::arg("threshold") = 0.7, py::arg("fanout") = 3, py::arg("group_mode") = 1,
           py::arg("use_graphs") = true, py::arg("device_refit") = true, py::arg("n_dom") = 10,
           py::arg("ttft_slo_ms") = 800.0f, py::arg("halo_ms") = 0.0, py::arg("import_cap") = 0,
           py::arg("xchg_cap") = 0, py::arg("shard_rank") = 0, py::arg("shard_world") = 1,
           py::arg("halo_windows") = 3, py::arg("split_rings") = false)
      .def("register_host", &PyEngine::register_host)
      .def("submit", &PyEngine::submit, py::arg("k"), py::arg("kernel"), py::arg("user"), py::arg("spans"),
           py::arg("n_groups"), py::arg("labels") = py::none(), py::arg("bases") = std::vector<int64_t>{},
           py::arg("with_labels") = true, py::arg("learn") = false, py::arg("user_rec") = 64)
      .def("h2d_done", &PyEngine::h2d_done)
      .def("wait_h2d", &PyEngine::wait_h2d)
      .def("query", &PyEngine::query)
      .def("wait", &PyEngine::wait)
      .def("packet", &PyEngine::packet)
      .def("results", &PyEngine::results)
      .def("window_ms", &PyEngine::window_ms)
      .def("copy_ms", [](PyEngine& p, int64_t k) {
        py::gil_scoped_release nogil;
        return p.eng().copy_ms(k);
      })
      .def("set_model_bytes", &PyEngine::set_model_bytes)
      .def("set_app_model", &PyEngine::set_app_model)
      .def("set_p0", &PyEngine::set_p0)
      .def("set_refit", &PyEngine::set_refit, py::arg("alpha") = 2.0, py::arg("prior_pseudo") = 1.0,
           py::arg("inv_temp") = 1.0, py::arg("min_count") = 0.0, py::arg("cap_dom") = -1, py::arg("ceil") = 1.0)
      .def("refit_now", &PyEngine::refit_now)
      .def("set_device_refit", [](PyEngine& p, bool on) { p.eng().set_device_refit(on); })
      .def("score", &PyEngine::score, py::arg("feat"), py::arg("labels") = py::none(), py::arg("app") = py::none())
      .def("set_pods", &PyEngine::set_pods)
      .def("inject_remote", &PyEngine::inject_remote)
      .def("results_all", &PyEngine::results_all)
      .def("set_join_params", &PyEngine::set_join_params)
      .def("init_comm", &PyEngine::init_comm)
      .def("totals", &PyEngine::totals)
      .def("reset_totals", &PyEngine::reset_totals)
      .def("stats_acc", &PyEngine::stats_acc)
      .def("model_bytes", &PyEngine::model_bytes)
      .def("restore", &PyEngine::restore)
      .def("sync", &PyEngine::sync)
      .def("import_state", &PyEngine::import_state)
      .def("sent_block", &PyEngine::sent_block)
      .def("close", &PyEngine::close)
      .def_property_readonly("buffers", &PyEngine::buffers)
      .def_property_readonly("windows_folded", &PyEngine::folded)
      .def_property_readonly("graphs", &PyEngine::graphs)
      .def_property_readonly("host_issue_us", &PyEngine::host_issue_us)
      .def_property_readonly("host_wait_us", &PyEngine::host_wait_us)
      .def_property_readonly("host_dma_issue_us", &PyEngine::host_dma_issue_us)
      .def_property_readonly("host_launch_us", &PyEngine::host_launch_us)
      .def_property_readonly("host_pre_us", [](PyEngine& p) { return p.eng().host_pre_us(); })
      .def_property_readonly("host_dma_split_us", [](PyEngine& p) { return p.eng().host_dma_split_us(); })
      .def_property_readonly("host_tail_us", [](PyEngine& p) { return p.eng().host_tail_us(); })
      .def_property_readonly("has_comm", &PyEngine::has_comm)
      .def_property_readonly("rank", [](PyEngine& p) { return p.eng().rank(); })
      .def_property_readonly("world", [](PyEngine& p) { return p.eng().world(); })
      .def_property_readonly("staged_bytes", &PyEngine::staged_bytes)
      .def_property_readonly("direct_bytes", &PyEngine::direct_bytes);
}
