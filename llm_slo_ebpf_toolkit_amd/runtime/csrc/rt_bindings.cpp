// pybind11 module `_mislo_rt`: the host runtime (ring, shared-memory rings, pinning for
// direct DMA, paced replay producers) for the Python agent / benchmark.
#include <hip/hip_runtime_api.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "replay.h"
#include "ring.h"
#include "wire.h"

namespace py = pybind11;
using mislo::Ring;

class HostRing {
 public:
  HostRing(uint64_t capacity, uint32_t rec_size, const std::string& shm_name) : shm_name_(shm_name) {
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
    unpin();
    if (shm_) {
      mislo_ring_close(shm_);
      mislo_ring_unlink_shm(shm_name_.c_str());
    } else {
      delete ring_;
      free(mem_);
    }
  }

  // Page-lock the record array so hipMemcpyAsync DMAs straight from the ring.
  bool pin() {
    if (pinned_) return true;
    const size_t n = ring_->capacity() * ring_->rec_size();
    pinned_ = hipHostRegister(ring_->records(), n, hipHostRegisterPortable) == hipSuccess;
    return pinned_;
  }
  void unpin() {
    if (pinned_) (void)hipHostUnregister(ring_->records());
    pinned_ = false;
  }

  uint64_t push(py::buffer b) {
    py::buffer_info info = b.request();
    const uint64_t nbytes = (uint64_t)info.size * info.itemsize;
    if (nbytes % ring_->rec_size()) throw std::invalid_argument("buffer is not a whole number of records");
    const uint64_t n = nbytes / ring_->rec_size();
    py::gil_scoped_release nogil;
    return ring_->push_batch(info.ptr, n);
  }

  py::list peek(uint64_t max_records) {
    mislo::Segment seg[2];
    int ns = ring_->peek(max_records, seg);
    py::list out;
    for (int i = 0; i < ns; ++i) out.append(py::make_tuple(seg[i].pos, seg[i].index, seg[i].count));
    return out;
  }

  void release(uint64_t n) { ring_->release(n); }
  uint64_t size() const { return ring_->size(); }
  uint64_t capacity() const { return ring_->capacity(); }
  uint32_t rec_size() const { return ring_->rec_size(); }
  uintptr_t address() const { return reinterpret_cast<uintptr_t>(ring_->records()); }
  bool pinned() const { return pinned_; }

  py::array records_view() {
    return py::array(py::dtype("uint8"), {(py::ssize_t)(ring_->capacity() * ring_->rec_size())},
                     {(py::ssize_t)1}, ring_->records(), py::cast(this, py::return_value_policy::reference));
  }

  // Async H2D of `count` records starting at slot `index` to device address `dst` on `stream`.
  void copy_to_device(uintptr_t dst, uint64_t index, uint64_t count, uintptr_t stream) {
    if (index + count > ring_->capacity()) throw std::out_of_range("segment past ring end");
    const size_t rs = ring_->rec_size();
    hipError_t e = hipMemcpyAsync(reinterpret_cast<void*>(dst), ring_->records() + index * rs, count * rs,
                                  hipMemcpyHostToDevice, reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) throw std::runtime_error(std::string("hipMemcpyAsync: ") + hipGetErrorString(e));
  }

  py::dict stats() const {
    auto* h = ring_->header();
    py::dict d;
    d["pushed"] = h->pushed.load();
    d["dropped"] = h->dropped.load();
    d["high_water"] = h->high_water.load();
    d["batches"] = h->batches.load();
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
  bool pinned_ = false;
};

class PyReplayer {
 public:
  PyReplayer(HostRing& ring, py::buffer trace, int64_t lap_ns) {
    py::buffer_info info = trace.request();
    const uint64_t nbytes = (uint64_t)info.size * info.itemsize;
    const uint32_t rs = ring.rec_size();
    if (nbytes % rs || nbytes == 0) throw std::invalid_argument("trace is not a whole number of records");
    rep_ = std::make_unique<mislo::Replayer>(ring.ring(), reinterpret_cast<const uint8_t*>(info.ptr), nbytes / rs, rs,
                                             lap_ns);
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
  std::unique_ptr<mislo::Replayer> rep_;
};

// 64-byte EVENT / SPAN records -> 20- or 16-byte wire records (runtime/csrc/wire.h)
class PyWireEncoder {
 public:
  explicit PyWireEncoder(py::array_t<int8_t, py::array::c_style | py::array::forcecast> shift) {
    if (shift.size() != 256) throw std::invalid_argument("shift must have 256 entries");
    enc_ = std::make_unique<mislo::WireEncoder>(shift.data());
  }

  // events: EVENT records (any contiguous buffer, n*64 bytes); out: writable buffer of
  // >= n*wire bytes (e.g. the pinned staging tensor). Returns t_base.
  int64_t encode(py::buffer events, py::buffer out, int wire) {
    py::buffer_info ei = events.request(), oi = out.request(true);
    const size_t nb = (size_t)ei.size * ei.itemsize;
    if (nb % sizeof(mislo::EventRec)) throw std::invalid_argument("events: not a whole number of 64-byte records");
    const size_t n = nb / sizeof(mislo::EventRec);
    if ((size_t)oi.size * oi.itemsize < n * (size_t)mislo::wire_bytes(wire))
      throw std::invalid_argument("out buffer too small");
    py::gil_scoped_release nogil;
    return enc_->encode(static_cast<const mislo::EventRec*>(ei.ptr), n, oi.ptr, wire);
  }

  // spans -> 20-byte SPAN20 records (out >= n*20 bytes)
  void encode_spans20(py::buffer spans, py::buffer out) {
    py::buffer_info si = spans.request(), oi = out.request(true);
    const size_t nb = (size_t)si.size * si.itemsize;
    if (nb % sizeof(mislo::SpanRec64)) throw std::invalid_argument("spans: not a whole number of 64-byte records");
    const size_t n = nb / sizeof(mislo::SpanRec64);
    if ((size_t)oi.size * oi.itemsize < n * sizeof(mislo::Span20)) throw std::invalid_argument("out buffer too small");
    py::gil_scoped_release nogil;
    enc_->encode_spans20(static_cast<const mislo::SpanRec64*>(si.ptr), n, static_cast<mislo::Span20*>(oi.ptr));
  }

  void encode_spans(py::buffer spans, py::buffer out, bool trace_ids) {
    py::buffer_info si = spans.request(), oi = out.request(true);
    const size_t nb = (size_t)si.size * si.itemsize;
    if (nb % sizeof(mislo::SpanRec64)) throw std::invalid_argument("spans: not a whole number of 64-byte records");
    if ((size_t)oi.size * oi.itemsize < nb) throw std::invalid_argument("out buffer too small");
    py::gil_scoped_release nogil;
    enc_->encode_spans(static_cast<const mislo::SpanRec64*>(si.ptr), nb / sizeof(mislo::SpanRec64),
                       static_cast<mislo::SpanRec64*>(oi.ptr), trace_ids);
  }

  // one window on the worker pool (wire.h encode_window): events -> ev_out, spans -> sp_out
  int64_t encode_window(py::buffer events, py::buffer ev_out, int wire, py::buffer spans, py::buffer sp_out,
                        int threads, size_t min_chunk) {
    py::buffer_info ei = events.request(), eo = ev_out.request(true), si = spans.request(), so = sp_out.request(true);
    const size_t nb = (size_t)ei.size * ei.itemsize, sb = (size_t)si.size * si.itemsize;
    if (nb % sizeof(mislo::EventRec)) throw std::invalid_argument("events: not a whole number of 64-byte records");
    if (sb % sizeof(mislo::SpanRec64)) throw std::invalid_argument("spans: not a whole number of 64-byte records");
    const size_t n = nb / sizeof(mislo::EventRec), ns = sb / sizeof(mislo::SpanRec64);
    if ((size_t)eo.size * eo.itemsize < n * (size_t)wire) throw std::invalid_argument("ev_out buffer too small");
    if ((size_t)so.size * so.itemsize < sb) throw std::invalid_argument("sp_out buffer too small");
    py::gil_scoped_release nogil;
    return enc_->encode_window(static_cast<const mislo::EventRec*>(ei.ptr), n, eo.ptr, wire,
                               static_cast<const mislo::SpanRec64*>(si.ptr), ns,
                               static_cast<mislo::SpanRec64*>(so.ptr), threads, min_chunk);
  }

  void end_window() { enc_->end_window(); }

  // context table (int32 [n, 4]: pod, pid, conn id, svc<<16|node), row i = context id i
  py::array_t<int32_t> ctx_table() const {
    const auto& rows = enc_->ctx_rows();
    py::array_t<int32_t> a({(py::ssize_t)rows.size(), (py::ssize_t)4});
    std::memcpy(a.mutable_data(), rows.data(), rows.size() * sizeof(rows[0]));
    return a;
  }
  size_t n_ctx() const { return enc_->ctx_rows().size(); }
  size_t n_conns() const { return enc_->n_conns(); }
  size_t n_traces() const { return enc_->n_traces(); }

 private:
  std::unique_ptr<mislo::WireEncoder> enc_;
};

PYBIND11_MODULE(_mislo_rt, m) {
  m.doc() = "MI355X LLM-SLO native host runtime (rings, replay producers)";
  py::class_<HostRing>(m, "HostRing")
      .def(py::init<uint64_t, uint32_t, const std::string&>(), py::arg("capacity"), py::arg("rec_size") = 64,
           py::arg("shm_name") = "")
      .def("pin", &HostRing::pin)
      .def("unpin", &HostRing::unpin)
      .def("push", &HostRing::push)
      .def("peek", &HostRing::peek)
      .def("release", &HostRing::release)
      .def("records_view", &HostRing::records_view)
      .def("copy_to_device", &HostRing::copy_to_device)
      .def("stats", &HostRing::stats)
      .def_property_readonly("size", &HostRing::size)
      .def_property_readonly("capacity", &HostRing::capacity)
      .def_property_readonly("rec_size", &HostRing::rec_size)
      .def_property_readonly("address", &HostRing::address)
      .def_property_readonly("pinned", &HostRing::pinned);
  py::class_<PyReplayer>(m, "Replayer")
      .def(py::init<HostRing&, py::buffer, int64_t>(), py::arg("ring"), py::arg("trace"), py::arg("lap_ns"),
           py::keep_alive<1, 2>())
      .def("start", &PyReplayer::start, py::arg("threads") = 1, py::arg("rate_eps") = 0.0,
           py::arg("batch") = 256, py::arg("max_records") = 0)
      .def("stop", &PyReplayer::stop)
      .def("wait", &PyReplayer::wait)
      .def_property_readonly("pushed", &PyReplayer::pushed)
      .def_property_readonly("dropped", &PyReplayer::dropped);
  py::class_<PyWireEncoder>(m, "WireEncoder")
      .def(py::init<py::array_t<int8_t, py::array::c_style | py::array::forcecast>>(), py::arg("shift"))
      .def("encode", &PyWireEncoder::encode, py::arg("events"), py::arg("out"), py::arg("wire") = 20)
      .def("encode_spans20", &PyWireEncoder::encode_spans20, py::arg("spans"), py::arg("out"))
      .def("encode_spans", &PyWireEncoder::encode_spans, py::arg("spans"), py::arg("out"),
           py::arg("trace_ids") = false)
      .def("encode_window", &PyWireEncoder::encode_window, py::arg("events"), py::arg("ev_out"), py::arg("wire"),
           py::arg("spans"), py::arg("sp_out"), py::arg("threads") = 8,
           py::arg("min_chunk") = 16384)
      .def("end_window", &PyWireEncoder::end_window)
      .def("ctx_table", &PyWireEncoder::ctx_table)
      .def_property_readonly("n_ctx", &PyWireEncoder::n_ctx)
      .def_property_readonly("n_conns", &PyWireEncoder::n_conns)
      .def_property_readonly("n_traces", &PyWireEncoder::n_traces);
}
