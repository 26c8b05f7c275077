// pybind11 module `_mislo_rt`: the agent's host runtime (CPU only: no HIP runtime in this
// module, so a process loads exactly one HIP runtime -- the engine's, or PyTorch's). Shared-memory MPSC rings for
// user-space producers, the BPF ring buffer view / consumer / kernel-probe model, the agent's
// id tables and window assembler, bpf(2) map access, paced replay producers.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <errno.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "assemble.h"
#include "bpfring.h"
#include "bpfsys.h"
#include "probesim.h"
#include "gpusampler.h"
#include "procsampler.h"
#include "replay.h"
#include "ring.h"
#include "tables.h"

namespace py = pybind11;
using namespace mislo;

namespace {

template <class T>
std::pair<const T*, size_t> records_of(const py::buffer& b, const char* what) {
  py::buffer_info info = b.request();
  const size_t nb = (size_t)info.size * info.itemsize;
  if (nb % sizeof(T)) throw std::invalid_argument(std::string(what) + ": not a whole number of records");
  return {static_cast<const T*>(info.ptr), nb / sizeof(T)};
}

py::array_t<uint32_t> rec16_array(const Rec16* r, size_t n) {
  py::array_t<uint32_t> a({(py::ssize_t)n, (py::ssize_t)4});
  if (n) std::memcpy(a.mutable_data(), r, n * sizeof(Rec16));
  return a;
}

const int8_t* shift_of(const py::array_t<int8_t, py::array::c_style | py::array::forcecast>& shift) {
  if (shift.size() != 256) throw std::invalid_argument("shift must have 256 entries");
  return shift.data();
}

py::dict layout_dict(const SlotLayout& L) {
  py::dict d;
  d["group_cap"] = L.group_cap;
  d["span_cap"] = L.span_cap;
  d["sig_cap"] = L.sig_cap;
  d["row_cap"] = L.row_cap;
  d["sp_off"] = L.sp_off;
  d["ev_off"] = L.ev_off;
  d["bytes"] = L.bytes;
  return d;
}

}  // namespace

class HostRing {
 public:
  HostRing(uint64_t capacity, uint32_t rec_size, const std::string& shm_name, bool attach) : shm_name_(shm_name) {
    if (attach) {
      shm_ = mislo_ring_open_shm(shm_name.c_str());
      if (!shm_) throw std::runtime_error("cannot attach shared-memory ring " + shm_name);
      ring_ = static_cast<Ring*>(mislo_ring_handle_ring(shm_));
      owner_ = false;
      return;
    }
    if (capacity == 0 || (capacity & (capacity - 1))) throw std::invalid_argument("capacity must be a power of two");
    if (!shm_name.empty()) {
      shm_ = mislo_ring_create_shm(shm_name.c_str(), capacity, rec_size);
      if (!shm_) throw std::runtime_error("cannot create shared-memory ring " + shm_name);
      ring_ = static_cast<Ring*>(mislo_ring_handle_ring(shm_));
    } else {
      bytes_ = Ring::bytes_for(capacity, rec_size);
      if (posix_memalign(&mem_, 4096, bytes_) != 0) throw std::bad_alloc();
      std::memset(mem_, 0, bytes_);
      ring_ = Ring::format(mem_, capacity, rec_size);
    }
    if (!ring_) throw std::runtime_error("ring format failed");
  }
  ~HostRing() {
    if (shm_) {
      mislo_ring_close(shm_);
      if (owner_) mislo_ring_unlink_shm(shm_name_.c_str());
    } else {
      delete ring_;
      free(mem_);
    }
  }

  uint64_t push(py::buffer b, int threads) {
    py::buffer_info info = b.request();
    const uint64_t nbytes = (uint64_t)info.size * info.itemsize;
    if (nbytes % ring_->rec_size()) throw std::invalid_argument("buffer is not a whole number of records");
    const uint64_t n = nbytes / ring_->rec_size();
    py::gil_scoped_release nogil;
    return ring_->push_batch(info.ptr, n, threads);
  }

  py::list peek(uint64_t max_records) {
    Segment seg[2];
    int ns = ring_->peek(max_records, seg);
    py::list out;
    for (int i = 0; i < ns; ++i) out.append(py::make_tuple(seg[i].pos, seg[i].index, seg[i].count));
    return out;
  }

  void release(uint64_t n) { ring_->release(n); }
  uint64_t size() const { return ring_->size(); }
  uint64_t capacity() const { return ring_->capacity(); }
  uint32_t rec_size() const { return ring_->rec_size(); }
  uint64_t head() const { return ring_->header()->head.load(std::memory_order_acquire); }
  uint64_t tail() const { return ring_->header()->tail.load(std::memory_order_acquire); }
  uintptr_t address() const { return reinterpret_cast<uintptr_t>(ring_->records()); }
  uint32_t drop_mask() const { return ring_->header()->drop_mask.load(std::memory_order_relaxed); }
  void set_drop_mask(uint32_t m) { ring_->header()->drop_mask.store(m, std::memory_order_relaxed); }

  py::array records_view() {
    return py::array(py::dtype("uint8"), {(py::ssize_t)(ring_->capacity() * ring_->rec_size())}, {(py::ssize_t)1},
                     ring_->records(), py::cast(this, py::return_value_policy::reference));
  }

  py::dict stats() const {
    auto* h = ring_->header();
    py::dict d;
    d["pushed"] = h->pushed.load();
    d["dropped"] = h->dropped.load();
    d["high_water"] = h->high_water.load();
    d["batches"] = h->batches.load();
    d["stolen"] = h->stolen.load();
    d["size"] = ring_->size();
    d["capacity"] = ring_->capacity();
    return d;
  }

  Ring* ring() { return ring_; }

 private:
  std::string shm_name_;
  void* shm_ = nullptr;
  void* mem_ = nullptr;
  size_t bytes_ = 0;
  Ring* ring_ = nullptr;
  bool owner_ = true;
};

class PyReplayer {
 public:
  PyReplayer(HostRing& ring, py::buffer trace, int64_t lap_ns) {
    py::buffer_info info = trace.request();
    const uint64_t nbytes = (uint64_t)info.size * info.itemsize;
    const uint32_t rs = ring.rec_size();
    if (nbytes % rs || nbytes == 0) throw std::invalid_argument("trace is not a whole number of records");
    rep_ = std::make_unique<Replayer>(ring.ring(), reinterpret_cast<const uint8_t*>(info.ptr), nbytes / rs, rs, lap_ns);
  }
  void start(int threads, double rate_eps, uint64_t batch, uint64_t max_records) {
    rep_->start(threads, rate_eps, batch, max_records);
  }
  void stop() {
    py::gil_scoped_release nogil;
    rep_->stop();
  }
  void wait() {
    py::gil_scoped_release nogil;
    rep_->wait();
  }
  uint64_t pushed() const { return rep_->pushed(); }
  uint64_t dropped() const { return rep_->dropped(); }

 private:
  std::unique_ptr<Replayer> rep_;
};

// ---- BPF ring buffer ----------------------------------------------------------------------

class PyRingbuf {
 public:
  explicit PyRingbuf(std::unique_ptr<Ringbuf> rb, int fd = -1) : rb_(std::move(rb)), fd_(fd) {}
  ~PyRingbuf() {
    rb_.reset();
    if (fd_ >= 0) ::close(fd_);
  }
  static std::unique_ptr<PyRingbuf> create_shm(const std::string& name, uint64_t size) {
    return std::make_unique<PyRingbuf>(Ringbuf::create_shm(name, size));
  }
  static std::unique_ptr<PyRingbuf> attach_shm(const std::string& name) {
    return std::make_unique<PyRingbuf>(Ringbuf::attach_shm(name));
  }
  // a pinned BPF ringbuf map (/sys/fs/bpf/.../mislo_events)
  static std::unique_ptr<PyRingbuf> open_pinned(const std::string& path) {
    const int fd = bpf_obj_get(path);
    if (fd < 0) throw std::runtime_error("BPF_OBJ_GET " + path + ": " + std::strerror(-fd));
    BpfMapInfo info;
    const int r = bpf_map_info(fd, &info);
    if (r < 0) {
      ::close(fd);
      throw std::runtime_error("BPF_OBJ_GET_INFO_BY_FD: " + std::string(std::strerror(-r)));
    }
    if (info.type != 27 /* BPF_MAP_TYPE_RINGBUF */) {
      ::close(fd);
      throw std::runtime_error(path + " is not a BPF ring buffer map");
    }
    return std::make_unique<PyRingbuf>(Ringbuf::open_map_fd(fd, info.max_entries), fd);
  }
  Ringbuf* rb() { return rb_.get(); }
  uint64_t cfg_get(int i) const {
    check_cfg(i);
    return __atomic_load_n(&rb_->cfg()[i], __ATOMIC_ACQUIRE);
  }
  void cfg_set(int i, uint64_t v) {
    check_cfg(i);
    __atomic_store_n(&rb_->cfg()[i], v, __ATOMIC_RELEASE);
  }
  bool output(py::buffer b) {
    py::buffer_info info = b.request();
    return rb_->output(info.ptr, (uint32_t)(info.size * info.itemsize));
  }
  uintptr_t reserve(uint32_t size) { return reinterpret_cast<uintptr_t>(rb_->reserve(size)); }
  void write(uintptr_t at, py::buffer b) {
    py::buffer_info info = b.request();
    std::memcpy(reinterpret_cast<void*>(at), info.ptr, (size_t)(info.size * info.itemsize));
  }
  void commit(uintptr_t at, bool discard) { rb_->commit(reinterpret_cast<void*>(at), discard); }
  bool append_framed(py::buffer b, int threads) {
    py::buffer_info info = b.request();
    const uint8_t* p = static_cast<const uint8_t*>(info.ptr);
    const uint64_t n = (uint64_t)(info.size * info.itemsize);
    py::gil_scoped_release nogil;
    return rb_->append_framed(p, n, threads);
  }
  py::array data_view() {
    return py::array(py::dtype("uint8"), {(py::ssize_t)(2 * rb_->size())}, {(py::ssize_t)1}, rb_->data(),
                     py::cast(this, py::return_value_policy::reference));
  }
  void set_consumer_pos(uint64_t p) { rb_->set_consumer_pos(p); }
  py::dict stats() const {
    py::dict d;
    d["size"] = rb_->size();
    d["consumer_pos"] = rb_->consumer_pos();
    d["producer_pos"] = rb_->producer_pos();
    if (rb_->meta()) {
      d["dropped"] = rb_->meta()->dropped.load();
      d["reserved"] = rb_->meta()->reserved.load();
    }
    return d;
  }

 private:
  void check_cfg(int i) const {
    if (!rb_->cfg()) throw std::logic_error("mislo_cfg of a real ring lives in its own BPF map (BpfMap)");
    if (i < 0 || i >= kCfgSlots) throw std::out_of_range("cfg index");
  }
  std::unique_ptr<Ringbuf> rb_;
  int fd_;
};

class PyConsumer {
 public:
  PyConsumer(PyRingbuf& rb, int threads) : c_(rb.rb(), threads) {}
  py::tuple consume(py::buffer out, uint64_t cap, uint64_t limit) {
    py::buffer_info oi = out.request(true);
    if ((uint64_t)(oi.size * oi.itemsize) < cap * sizeof(Rec16)) throw std::invalid_argument("out buffer too small");
    std::vector<Rec16> defs;
    ConsumeStats st;
    {
      py::gil_scoped_release nogil;
      st = c_.consume(static_cast<Rec16*>(oi.ptr), cap, defs, limit);
    }
    py::dict d;
    d["events"] = st.events;
    d["defs"] = st.defs;
    d["pads"] = st.pads;
    d["discarded"] = st.discarded;
    d["foreign"] = st.foreign;
    d["begin_pos"] = st.begin_pos;
    d["end_pos"] = st.end_pos;
    d["busy_stop"] = st.busy_stop;
    d["serial"] = st.serial;
    return py::make_tuple(d, rec16_array(defs.data(), defs.size()));
  }
  RingbufConsumer* get() { return &c_; }
  int threads() const { return c_.threads(); }

 private:
  RingbufConsumer c_;
};

class PyProbeSim {
 public:
  PyProbeSim(PyRingbuf& rb, py::array_t<int8_t, py::array::c_style | py::array::forcecast> shift, size_t trace_lru,
             uint32_t cpus)
      : rb_(rb), sim_(rb.rb()->cfg(), shift_of(shift), trace_lru, cpus) {}
  uint64_t submit(py::buffer events, bool flush) {
    auto [ev, n] = records_of<EventRec>(events, "events");
    py::gil_scoped_release nogil;
    return sim_.submit(*rb_.rb(), ev, n, flush);
  }
  uint64_t flush() {
    py::gil_scoped_release nogil;
    return sim_.flush(*rb_.rb());
  }
  py::array_t<uint32_t> encode(py::buffer events, bool flush) {
    auto [ev, n] = records_of<EventRec>(events, "events");
    std::vector<Rec16> out;
    {
      py::gil_scoped_release nogil;
      sim_.encode(ev, n, out, flush);
    }
    return rec16_array(out.data(), out.size());
  }
  py::array_t<uint32_t> encode_flush() {
    std::vector<Rec16> out;
    sim_.encode_flush(out);
    return rec16_array(out.data(), out.size());
  }
  uint64_t batches() const { return sim_.batches(); }
  void reset_maps() { sim_.reset_maps(); }
  size_t n_ctx() const { return sim_.n_ctx(); }
  size_t n_traces() const { return sim_.n_traces(); }
  uint64_t dropped() const { return sim_.dropped(); }

 private:
  PyRingbuf& rb_;
  ProbeSim sim_;
};

py::array_t<uint8_t> frame_records_py(py::buffer recs) {
  auto [r, n] = records_of<Rec16>(recs, "records");
  if (n % kBatchSlots) throw std::invalid_argument("frame_records: whole batches of 8 slots only");
  py::array_t<uint8_t> out((py::ssize_t)(n / kBatchSlots * kRecStride));
  frame_records(r, n, out.mutable_data());
  return out;
}

class PyTables {
 public:
  explicit PyTables(py::array_t<int8_t, py::array::c_style | py::array::forcecast> shift) : t_(shift_of(shift)) {}
  void set_pod(uint32_t pod, uint32_t sn) { t_.set_pod(pod, sn); }
  void set_pods(py::array_t<uint32_t, py::array::c_style | py::array::forcecast> pods,
                py::array_t<uint32_t, py::array::c_style | py::array::forcecast> sn) {
    if (pods.size() != sn.size()) throw std::invalid_argument("pods / svcnode size mismatch");
    for (py::ssize_t i = 0; i < pods.size(); ++i) t_.set_pod(pods.data()[i], sn.data()[i]);
  }
  uint32_t pod_svcnode(uint32_t pod) const { return t_.pod_svcnode(pod); }
  void apply_defs(py::buffer defs) {
    auto [d, n] = records_of<Rec16>(defs, "defs");
    t_.apply_defs(d, n);
  }
  py::array_t<uint32_t> encode_events(py::buffer events, std::vector<int64_t> bases) {
    auto [ev, n] = records_of<EventRec>(events, "events");
    if (bases.size() > 4) throw std::invalid_argument("at most 4 epoch bases");
    bases.resize(4, 0);
    std::vector<Rec16> out(n);
    t_.encode_events(ev, n, out.data(), bases.data());
    return rec16_array(out.data(), n);
  }
  py::array_t<uint8_t> encode_spans(py::buffer spans) {
    auto [sp, n] = records_of<SpanRec64>(spans, "spans");
    py::array_t<uint8_t> out((py::ssize_t)(n * sizeof(Span20)));
    t_.encode_spans(sp, n, reinterpret_cast<Span20*>(out.mutable_data()));
    return out;
  }
  uint32_t trace_id(uint64_t h) { return t_.trace_id(h); }
  void set_sli_threshold(float ms) { t_.set_sli_threshold(ms); }
  py::array_t<uint32_t> take_group_sli(size_t groups) {
    py::array_t<uint32_t> a({(py::ssize_t)groups, (py::ssize_t)2});
    std::vector<uint32_t> n(groups), b(groups);
    t_.take_group_sli(n.data(), b.data(), groups);
    auto m = a.mutable_unchecked<2>();
    for (size_t g = 0; g < groups; ++g) {
      m(g, 0) = n[g];
      m(g, 1) = b[g];
    }
    return a;
  }
  py::tuple take_rows(size_t cap) {
    std::vector<uint32_t> ids(cap);
    std::vector<AgentTables::Row> rows(cap);
    const size_t k = t_.take_rows(ids.data(), rows.data(), cap);
    py::array_t<uint32_t> a((py::ssize_t)k), b({(py::ssize_t)k, (py::ssize_t)4});
    if (k) {
      std::memcpy(a.mutable_data(), ids.data(), 4 * k);
      std::memcpy(b.mutable_data(), rows.data(), 16 * k);
    }
    return py::make_tuple(a, b);
  }
  void end_window() { t_.end_window(); }
  AgentTables* get() { return &t_; }
  py::dict stats() const {
    py::dict d;
    d["kernel_ctx"] = t_.n_kernel_ctx();
    d["host_ctx"] = t_.n_host_ctx();
    d["traces"] = t_.n_traces();
    d["pending_rows"] = t_.pending_rows();
    d["host_ctx_wraps"] = t_.host_ctx_wraps();
    d["bad_defs"] = t_.bad_defs();
    return d;
  }

 private:
  AgentTables t_;
};

class PyAssembler {
 public:
  PyAssembler(uint32_t group_cap, uint32_t span_cap, uint32_t sig_cap, uint32_t row_cap, PyTables& tables,
              PyConsumer* kernel, HostRing* user, HostRing* spans)
      : a_(slot_layout(group_cap, span_cap, sig_cap, row_cap), tables.get(), kernel ? kernel->get() : nullptr,
           user ? user->ring() : nullptr, spans ? spans->ring() : nullptr) {}
  py::dict assemble(uintptr_t slot, std::vector<int64_t> bases, int n_groups, py::object labels, uint64_t kernel_limit,
                    uint64_t user_limit, uint64_t span_limit) {
    bases.resize(4, 0);
    std::vector<int32_t> lab;
    if (!labels.is_none()) {
      auto arr = labels.cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
      lab.assign(arr.data(), arr.data() + arr.size());
      if ((int)lab.size() < n_groups) lab.resize(n_groups, -1);
    }
    AssembleResult r;
    {
      py::gil_scoped_release nogil;
      r = a_.assemble(reinterpret_cast<uint8_t*>(slot), bases.data(), n_groups, lab.empty() ? nullptr : lab.data(),
                      kernel_limit, user_limit, span_limit);
    }
    py::dict d;
    d["n_events"] = r.n_events;
    d["n_kernel"] = r.n_kernel;
    d["n_user"] = r.n_user;
    d["n_spans"] = r.n_spans;
    d["n_rows"] = r.n_rows;
    d["n_defs"] = r.n_defs;
    d["rows_deferred"] = r.rows_deferred;
    d["discarded"] = r.discarded;
    d["foreign"] = r.foreign;
    d["busy_stop"] = r.busy_stop;
    d["ring_begin"] = r.ring_begin;
    d["ring_end"] = r.ring_end;
    d["user_dropped"] = r.user_dropped;
    d["dma_bytes"] = r.dma_bytes;
    d["host_us"] = r.host_us;
    return d;
  }
  py::dict layout() const { return layout_dict(a_.layout()); }

 private:
  WindowAssembler a_;
};

// procsampler.h: the agent's native schedstat / cgroup / PSI sampler thread, pushing into a user ring.
class PyProcSampler {
 public:
  PyProcSampler(HostRing* ring, uint32_t node_id, const std::string& proc_root, const std::string& cgroup_root,
                bool cgroup_cpu_psi, uint64_t runq_floor_ns, uint64_t steal_floor_milli, uint64_t cfs_floor_ns,
                uint64_t mem_floor_ns, uint32_t steal_sustain, uint64_t steal_foreign_milli,
                uint32_t steal_foreign_max_cpus) {
    ProcSamplerConfig c;
    c.node_id = node_id;
    c.proc_root = proc_root;
    c.cgroup_root = cgroup_root;
    c.cgroup_cpu_psi = cgroup_cpu_psi;
    c.runq_floor_ns = runq_floor_ns;
    c.steal_floor_milli = steal_floor_milli;
    c.cfs_floor_ns = cfs_floor_ns;
    c.mem_floor_ns = mem_floor_ns;
    c.steal_sustain = steal_sustain;
    c.steal_foreign_milli = steal_foreign_milli;
    c.steal_foreign_max_cpus = steal_foreign_max_cpus;
    s_ = std::make_unique<ProcSampler>(ring ? ring->ring() : nullptr, c);
  }
  void set_targets(const std::map<uint32_t, uint32_t>& pid_pod) {
    std::vector<std::pair<uint32_t, uint32_t>> v(pid_pod.begin(), pid_pod.end());
    s_->set_targets(v);
  }
  void set_target_list(const std::vector<std::pair<uint32_t, uint32_t>>& v) { s_->set_targets(v); }
  py::bytes tick(int64_t wall_ns, uint64_t mono_ns) {
    std::vector<EventRec> r;
    {
      py::gil_scoped_release nogil;
      r = s_->tick(wall_ns, mono_ns);
    }
    return py::bytes(reinterpret_cast<const char*>(r.data()), r.size() * sizeof(EventRec));
  }
  void start(double interval_s) {
    if (!(interval_s > 0)) throw std::invalid_argument("interval must be > 0");
    s_->start((uint64_t)(interval_s * 1e9));
  }
  void stop() {
    py::gil_scoped_release nogil;
    s_->stop();
  }
  uint32_t mask() const { return s_->mask(); }
  void set_mask(uint32_t m) { s_->set_mask(m); }
  bool paused() const { return s_->paused(); }
  void set_paused(bool p) { s_->set_paused(p); }
  py::dict stats() {
    ProcSamplerStats st = s_->stats();
    py::dict d;
    d["ticks"] = st.ticks;
    d["emitted"] = st.emitted;
    d["dropped"] = st.dropped;
    d["targets"] = st.targets;
    d["last_tick_ns"] = st.last_tick_ns;
    d["max_tick_ns"] = st.max_tick_ns;
    d["runqueue_delay_ms"] = st.by_type[0];
    d["cpu_steal_pct"] = st.by_type[1];
    d["mem_reclaim_latency_ms"] = st.by_type[2];
    d["cfs_throttled_ms"] = st.by_type[3];
    d["cfs_groups"] = st.cfs_groups;
    d["steal_gated"] = st.steal_gated;
    return d;
  }

 private:
  std::unique_ptr<ProcSampler> s_;
};

// gpusampler.h: the agent's KFD occupancy / eviction sampler thread, pushing into a user ring.
class PyGpuSampler {
 public:
  PyGpuSampler(HostRing* ring, uint32_t node_id, const std::string& kfd_proc, const std::string& proc_root,
               uint64_t floor_pct, uint64_t min_samples, uint64_t evict_floor_ns, bool evictions,
               uint32_t starved_hold, uint64_t starved_pct, uint32_t stamps) {
    GpuSamplerConfig c;
    c.stamps = stamps;
    c.starved_hold = starved_hold;
    c.starved_pct = starved_pct;
    c.node_id = node_id;
    c.kfd_proc = kfd_proc;
    c.proc_root = proc_root;
    c.floor_pct = floor_pct;
    c.min_samples = min_samples;
    c.evict_floor_ns = evict_floor_ns;
    c.evictions = evictions;
    s_ = std::make_unique<GpuSampler>(ring ? ring->ring() : nullptr, c);
  }
  void set_target_list(const std::vector<std::pair<uint32_t, uint32_t>>& v) {
    py::gil_scoped_release nogil;
    s_->set_targets(v);
  }
  void set_hip_map(int fd) { s_->set_hip_map(fd); }
  void set_hip_activity(uint32_t pid, uint64_t launches, uint64_t copies, uint64_t sync_ns, uint64_t syncs,
                        uint64_t copy_ns, uint64_t wait_ns, uint64_t waits) {
    HipActivity a;
    a.launches = launches, a.copies = copies, a.sync_ns = sync_ns, a.syncs = syncs;
    a.copy_ns = copy_ns, a.wait_ns = wait_ns, a.waits = waits;
    s_->set_hip_activity(pid, a);
  }
  void sample() {
    py::gil_scoped_release nogil;
    s_->sample();
  }
  py::bytes decide(int64_t wall_ns, uint64_t mono_ns) {
    std::vector<EventRec> r;
    {
      py::gil_scoped_release nogil;
      r = s_->decide(wall_ns, mono_ns);
    }
    return py::bytes(reinterpret_cast<const char*>(r.data()), r.size() * sizeof(EventRec));
  }
  void start(double sample_s, double decide_s) {
    if (!(sample_s > 0) || !(decide_s >= sample_s)) throw std::invalid_argument("need 0 < sample_s <= decide_s");
    s_->start((uint64_t)(sample_s * 1e9), (uint64_t)(decide_s * 1e9));
  }
  void stop() {
    py::gil_scoped_release nogil;
    s_->stop();
  }
  uint32_t mask() const { return s_->mask(); }
  void set_mask(uint32_t m) { s_->set_mask(m); }
  bool paused() const { return s_->paused(); }
  void set_paused(bool p) { s_->set_paused(p); }
  py::dict stats() {
    GpuSamplerStats st = s_->stats();
    py::dict d;
    d["samples"] = st.samples;
    d["reads"] = st.reads;
    d["scans"] = st.scans;
    d["sample_ns"] = st.read_ns;
    d["max_sample_ns"] = st.max_sample_ns;
    d["decisions"] = st.decisions;
    d["emitted"] = st.emitted;
    d["dropped"] = st.dropped;
    d["evictions"] = st.evictions;
    d["pairs"] = st.pairs;
    return d;
  }
  py::list shares() {
    py::list out;
    for (const GpuShare& g : s_->shares()) {
      py::dict d;
      d["pod"] = g.pod;
      d["gpu_id"] = g.gpu_id;
      d["samples"] = g.samples;
      d["hot"] = g.hot;
      d["own_hot"] = g.own_hot;
      d["share"] = g.share;
      d["gpu_wait_ns"] = g.gpu_wait_ns;
      d["wait_reported"] = g.wait_reported;
      d["delay_ns"] = g.delay_ns;
      d["foreign_mean"] = g.foreign_mean;
      d["active"] = g.active;
      d["starved"] = g.starved;
      out.append(d);
    }
    return out;
  }

 private:
  std::unique_ptr<GpuSampler> s_;
};

class PyBpfMap {
 public:
  explicit PyBpfMap(const std::string& path) {
    fd_ = bpf_obj_get(path);
    if (fd_ < 0) throw std::runtime_error("BPF_OBJ_GET " + path + ": " + std::strerror(-fd_));
    const int r = bpf_map_info(fd_, &info_);
    if (r < 0) throw std::runtime_error("BPF_OBJ_GET_INFO_BY_FD: " + std::string(std::strerror(-r)));
  }
  ~PyBpfMap() {
    if (fd_ >= 0) ::close(fd_);
  }
  py::object lookup(py::bytes key) {
    std::string k = key;
    if (k.size() != info_.key_size) throw std::invalid_argument("key size");
    std::string v(info_.value_size, '\0');
    const int r = bpf_map_lookup(fd_, k.data(), v.data());
    if (r == -ENOENT) return py::none();
    if (r < 0) throw std::runtime_error(std::string("lookup: ") + std::strerror(-r));
    return py::bytes(v);
  }
  void update(py::bytes key, py::bytes value, uint64_t flags) {
    std::string k = key, v = value;
    if (k.size() != info_.key_size || v.size() != info_.value_size) throw std::invalid_argument("key/value size");
    const int r = bpf_map_update(fd_, k.data(), v.data(), flags);
    if (r < 0) throw std::runtime_error(std::string("update: ") + std::strerror(-r));
  }
  bool remove(py::bytes key) {
    std::string k = key;
    const int r = bpf_map_delete(fd_, k.data());
    if (r == -ENOENT) return false;
    if (r < 0) throw std::runtime_error(std::string("delete: ") + std::strerror(-r));
    return true;
  }
  // all entries, by BPF_MAP_LOOKUP_BATCH (next_key walk where batching is unsupported)
  py::tuple items() {
    const uint32_t ks = info_.key_size, vs = info_.value_size;
    std::string keys, vals;
    uint32_t chunk = 4096;
    std::string kb(ks * (size_t)chunk, '\0'), vb(vs * (size_t)chunk, '\0');
    std::string in(ks, '\0'), out(ks, '\0');
    bool first = true, batch_ok = true;
    for (;;) {
      uint32_t cnt = chunk;
      const int r = bpf_map_lookup_batch(fd_, first ? nullptr : in.data(), out.data(), kb.data(), vb.data(), &cnt);
      if (r < 0 && r != -ENOENT) {
        if (first && (r == -EINVAL || r == -ENOTSUPP_ || r == -EOPNOTSUPP)) batch_ok = false;
        else throw std::runtime_error(std::string("lookup_batch: ") + std::strerror(-r));
        break;
      }
      keys.append(kb.data(), (size_t)cnt * ks);
      vals.append(vb.data(), (size_t)cnt * vs);
      if (r == -ENOENT) break;
      in = out;
      first = false;
    }
    if (!batch_ok) {
      std::string cur(ks, '\0'), nxt(ks, '\0'), v(vs, '\0');
      const void* prev = nullptr;
      while (bpf_map_next_key(fd_, prev, nxt.data()) == 0) {
        if (bpf_map_lookup(fd_, nxt.data(), v.data()) == 0) {
          keys.append(nxt);
          vals.append(v);
        }
        cur = nxt;
        prev = cur.data();
      }
    }
    return py::make_tuple(py::bytes(keys), py::bytes(vals));
  }
  py::dict info() const {
    py::dict d;
    d["type"] = info_.type;
    d["id"] = info_.id;
    d["key_size"] = info_.key_size;
    d["value_size"] = info_.value_size;
    d["max_entries"] = info_.max_entries;
    d["name"] = info_.name;
    return d;
  }

 private:
  static constexpr int ENOTSUPP_ = 524;  // kernel-internal ENOTSUPP
  int fd_ = -1;
  BpfMapInfo info_{};
};

PYBIND11_MODULE(_mislo_rt, m) {
  m.doc() = "MI355X LLM-SLO agent host runtime (rings, BPF ringbuf consumer, id tables, window assembly)";
  py::class_<HostRing>(m, "HostRing")
      .def(py::init<uint64_t, uint32_t, const std::string&, bool>(), py::arg("capacity") = 1, py::arg("rec_size") = 64,
           py::arg("shm_name") = "", py::arg("attach") = false)
      .def("push", &HostRing::push, py::arg("records"), py::arg("threads") = 1)
      .def("peek", &HostRing::peek)
      .def("release", &HostRing::release)
      .def("records_view", &HostRing::records_view)
      .def("stats", &HostRing::stats)
      .def_property_readonly("size", &HostRing::size)
      .def_property_readonly("capacity", &HostRing::capacity)
      .def_property_readonly("rec_size", &HostRing::rec_size)
      .def_property_readonly("head", &HostRing::head)
      .def_property("drop_mask", &HostRing::drop_mask, &HostRing::set_drop_mask)
      .def_property_readonly("tail", &HostRing::tail)
      .def_property_readonly("address", &HostRing::address);
  py::class_<PyReplayer>(m, "Replayer")
      .def(py::init<HostRing&, py::buffer, int64_t>(), py::arg("ring"), py::arg("trace"), py::arg("lap_ns"),
           py::keep_alive<1, 2>())
      .def("start", &PyReplayer::start, py::arg("threads") = 1, py::arg("rate_eps") = 0.0, py::arg("batch") = 256,
           py::arg("max_records") = 0)
      .def("stop", &PyReplayer::stop)
      .def("wait", &PyReplayer::wait)
      .def_property_readonly("pushed", &PyReplayer::pushed)
      .def_property_readonly("dropped", &PyReplayer::dropped);
  py::class_<PyRingbuf>(m, "Ringbuf")
      .def_static("create_shm", &PyRingbuf::create_shm, py::arg("name"), py::arg("size"))
      .def_static("attach_shm", &PyRingbuf::attach_shm, py::arg("name"))
      .def_static("open_pinned", &PyRingbuf::open_pinned, py::arg("path"))
      .def("cfg_get", &PyRingbuf::cfg_get)
      .def("cfg_set", &PyRingbuf::cfg_set)
      .def("output", &PyRingbuf::output)
      .def("reserve", &PyRingbuf::reserve)
      .def("write", &PyRingbuf::write)
      .def("commit", &PyRingbuf::commit, py::arg("at"), py::arg("discard") = false)
      .def("append_framed", &PyRingbuf::append_framed, py::arg("image"), py::arg("threads") = 1)
      .def("data_view", &PyRingbuf::data_view)
      .def("set_consumer_pos", &PyRingbuf::set_consumer_pos)
      .def("stats", &PyRingbuf::stats)
      .def_property_readonly("size", [](PyRingbuf& r) { return r.rb()->size(); })
      .def_property_readonly("data_address", [](PyRingbuf& r) { return reinterpret_cast<uintptr_t>(r.rb()->data()); })
      .def_property_readonly("page", [](PyRingbuf& r) { return r.rb()->page(); })
      .def_property_readonly("emulated", [](PyRingbuf& r) { return r.rb()->emulated(); })
      .def_property_readonly("consumer_pos", [](PyRingbuf& r) { return r.rb()->consumer_pos(); })
      .def_property_readonly("producer_pos", [](PyRingbuf& r) { return r.rb()->producer_pos(); })
      .def_property_readonly("available", [](PyRingbuf& r) { return r.rb()->available(); });
  py::class_<PyConsumer>(m, "RingbufConsumer")
      .def(py::init<PyRingbuf&, int>(), py::arg("ring"), py::arg("threads") = 1, py::keep_alive<1, 2>())
      .def("consume", &PyConsumer::consume, py::arg("out"), py::arg("cap"), py::arg("limit") = ~0ull)
      .def_property_readonly("threads", &PyConsumer::threads);
  py::class_<PyProbeSim>(m, "ProbeSim")
      .def(py::init<PyRingbuf&, py::array_t<int8_t, py::array::c_style | py::array::forcecast>, size_t, uint32_t>(),
           py::arg("ring"), py::arg("shift"), py::arg("trace_lru") = 1u << 20, py::arg("cpus") = 16,
           py::keep_alive<1, 2>())
      .def("submit", &PyProbeSim::submit, py::arg("events"), py::arg("flush") = true)
      .def("flush", &PyProbeSim::flush)
      .def("encode", &PyProbeSim::encode, py::arg("events"), py::arg("flush") = true)
      .def("encode_flush", &PyProbeSim::encode_flush)
      .def_property_readonly("batches", &PyProbeSim::batches)
      .def("reset_maps", &PyProbeSim::reset_maps)
      .def_property_readonly("n_ctx", &PyProbeSim::n_ctx)
      .def_property_readonly("n_traces", &PyProbeSim::n_traces)
      .def_property_readonly("dropped", &PyProbeSim::dropped);
  m.def("frame_records", &frame_records_py, py::arg("records"));
  py::class_<PyTables>(m, "AgentTables")
      .def(py::init<py::array_t<int8_t, py::array::c_style | py::array::forcecast>>(), py::arg("shift"))
      .def("set_pod", &PyTables::set_pod)
      .def("set_pods", &PyTables::set_pods)
      .def("pod_svcnode", &PyTables::pod_svcnode)
      .def("apply_defs", &PyTables::apply_defs)
      .def("encode_events", &PyTables::encode_events, py::arg("events"), py::arg("bases"))
      .def("encode_spans", &PyTables::encode_spans)
      .def("trace_id", &PyTables::trace_id)
      .def("set_sli_threshold", &PyTables::set_sli_threshold)
      .def("take_group_sli", &PyTables::take_group_sli)
      .def("take_rows", &PyTables::take_rows, py::arg("cap") = 1u << 20)
      .def("end_window", &PyTables::end_window)
      .def("stats", &PyTables::stats);
  py::class_<PyAssembler>(m, "WindowAssembler")
      .def(py::init<uint32_t, uint32_t, uint32_t, uint32_t, PyTables&, PyConsumer*, HostRing*, HostRing*>(),
           py::arg("group_cap"), py::arg("span_cap"), py::arg("sig_cap"), py::arg("row_cap"), py::arg("tables"),
           py::arg("kernel") = nullptr, py::arg("user") = nullptr, py::arg("spans") = nullptr, py::keep_alive<1, 6>(),
           py::keep_alive<1, 7>(), py::keep_alive<1, 8>(), py::keep_alive<1, 9>())
      .def("assemble", &PyAssembler::assemble, py::arg("slot"), py::arg("bases"), py::arg("n_groups"),
           py::arg("labels") = py::none(), py::arg("kernel_limit") = ~0ull, py::arg("user_limit") = ~0ull,
           py::arg("span_limit") = ~0ull)
      .def_property_readonly("layout", &PyAssembler::layout);
  m.def("slot_layout", [](uint32_t g, uint32_t s, uint32_t n, uint32_t r) { return layout_dict(slot_layout(g, s, n, r)); },
        py::arg("group_cap"), py::arg("span_cap"), py::arg("sig_cap"), py::arg("row_cap"));
  py::class_<PyGpuSampler>(m, "GpuSampler")
      .def(py::init<HostRing*, uint32_t, const std::string&, const std::string&, uint64_t, uint64_t, uint64_t, bool,
                    uint32_t, uint64_t, uint32_t>(),
           py::arg("ring"), py::arg("node_id") = 0, py::arg("kfd_proc") = "/sys/class/kfd/kfd/proc",
           py::arg("proc_root") = "/proc", py::arg("floor_pct") = 10, py::arg("min_samples") = 3,
           py::arg("evict_floor_ns") = 1000000, py::arg("evictions") = true, py::arg("starved_hold") = 2,
           py::arg("starved_pct") = 90, py::arg("stamps") = 1, py::keep_alive<1, 2>())
      .def("set_target_list", &PyGpuSampler::set_target_list)
      .def("set_hip_map", &PyGpuSampler::set_hip_map)
      .def("set_hip_activity", &PyGpuSampler::set_hip_activity, py::arg("pid"), py::arg("launches"),
           py::arg("copies") = 0, py::arg("sync_ns") = 0, py::arg("syncs") = 0, py::arg("copy_ns") = 0,
           py::arg("wait_ns") = 0, py::arg("waits") = 0)
      .def("sample", &PyGpuSampler::sample)
      .def("decide", &PyGpuSampler::decide, py::arg("wall_ns"), py::arg("mono_ns"))
      .def("start", &PyGpuSampler::start, py::arg("sample_s"), py::arg("decide_s"))
      .def("stop", &PyGpuSampler::stop)
      .def("stats", &PyGpuSampler::stats)
      .def("shares", &PyGpuSampler::shares)
      .def_property("mask", &PyGpuSampler::mask, &PyGpuSampler::set_mask)
      .def_property("paused", &PyGpuSampler::paused, &PyGpuSampler::set_paused);
  py::class_<PyProcSampler>(m, "ProcSampler")
      .def(py::init<HostRing*, uint32_t, const std::string&, const std::string&, bool, uint64_t, uint64_t, uint64_t,
                    uint64_t, uint32_t, uint64_t, uint32_t>(),
           py::arg("ring"), py::arg("node_id") = 0, py::arg("proc_root") = "/proc",
           py::arg("cgroup_root") = "/sys/fs/cgroup", py::arg("cgroup_cpu_psi") = false,
           py::arg("runq_floor_ns") = 100000, py::arg("steal_floor_milli") = 20000, py::arg("cfs_floor_ns") = 100000,
           py::arg("mem_floor_ns") = 100000, py::arg("steal_sustain") = 3, py::arg("steal_foreign_milli") = 25000,
           py::arg("steal_foreign_max_cpus") = 32, py::keep_alive<1, 2>())
      .def("set_targets", &PyProcSampler::set_targets)
      .def("set_target_list", &PyProcSampler::set_target_list)
      .def("tick", &PyProcSampler::tick, py::arg("wall_ns"), py::arg("mono_ns"))
      .def("start", &PyProcSampler::start, py::arg("interval_s"))
      .def("stop", &PyProcSampler::stop)
      .def("stats", &PyProcSampler::stats)
      .def_property("mask", &PyProcSampler::mask, &PyProcSampler::set_mask)
      .def_property("paused", &PyProcSampler::paused, &PyProcSampler::set_paused);
  py::class_<PyBpfMap>(m, "BpfMap")
      .def(py::init<const std::string&>(), py::arg("path"))
      .def("lookup", &PyBpfMap::lookup)
      .def("update", &PyBpfMap::update, py::arg("key"), py::arg("value"), py::arg("flags") = 0)
      .def("delete", &PyBpfMap::remove)
      .def("items", &PyBpfMap::items)
      .def("info", &PyBpfMap::info);
  m.def("bpf_available", &bpf_syscall_available);
  m.def(
      "perf_uprobe_open",
      [](uint32_t pmu_type, uint32_t retprobe_bit, bool retprobe, const std::string& path, uint64_t offset, int pid) {
        return perf_uprobe_open(UprobeAttr{pmu_type, retprobe_bit, retprobe, path, offset, pid});
      },
      py::arg("pmu_type"), py::arg("retprobe_bit"), py::arg("retprobe"), py::arg("path"), py::arg("offset"),
      py::arg("pid") = -1, "perf_event_open of a uprobe; an fd or -errno");
  m.def("bpf_link_create_perf", &bpf_link_create_perf, py::arg("prog_fd"), py::arg("perf_fd"),
        "BPF_LINK_CREATE(prog, perf event); a link fd or -errno");
  m.def("bpf_map_find", &bpf_map_find, py::arg("name"), py::arg("value_size") = 0,
        "fd of the first loaded BPF map of that name (and value size), or -errno");
  m.def("bpf_obj_get", &bpf_obj_get, py::arg("path"), "BPF_OBJ_GET of a pinned object; an fd or -errno");
  m.def("close_fd", &close_fd);
  m.def("bpf_obj_get", [](const std::string& path) { return bpf_obj_get(path); }, py::arg("path"));
  m.def("bpf_prog_run_on_cpu", &bpf_prog_run_on_cpu, py::arg("prog_fd"), py::arg("cpu"),
        py::call_guard<py::gil_scoped_release>());
  m.attr("REC_STRIDE") = kRecStride;
  m.attr("BATCH_SLOTS") = kBatchSlots;
  m.attr("DEF_PAD") = kPad;
  m.attr("DEF_TRACE") = kDefTrace;
  m.attr("DEF_CTX") = kDefCtx;
  m.attr("KERNEL_CTX_LIMIT") = kKernelCtxLimit;
  m.attr("KERNEL_TRACE_LIMIT") = kKernelTraceLimit;
  m.attr("CFG_EPOCH") = kCfgEpoch;
  m.attr("CFG_TRACE_NEXT") = kCfgTraceNext;
  m.attr("CFG_CTX_NEXT") = kCfgCtxNext;
  m.attr("CFG_CLOCK") = kCfgClock;
  m.attr("CFG_NODE") = kCfgNode;
}
