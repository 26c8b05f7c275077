// rocprofiler-sdk tool library: the user-space GPU signal source of the MI355X agent.
//
// Loaded into an LLM workload (ROCP_TOOL_LIBRARIES=libmislo_rocprof.so, no root needed),
// it turns runtime activity into the four GPU signals of the catalogue and pushes them into
// the agent's shared-memory ring (runtime/csrc/ring.h C ABI) as the ring's record type: 64-byte
// EVENT or, in rings created with 32- or 24-byte records, USER32 / USER24 (collector/records.py;
// the value in fixed point by the probes' own rule, mislo_record.h mislo_milli; USER24 packs
// pid / type / pod id and keeps the timestamp's low 44 bits -- 3/8 of the PCIe bytes of EVENT):
//
//   type 13 gpu_queue_delay_ms   kernel dispatch: start - enqueue            (ns)
//   type 14 hbm_pressure_pct     live device allocations / HBM capacity     (milli-pct)
//   type 15 xgmi_link_latency_us peer GPU copy time beyond its bytes at the
//                                link's nominal rate (the latency component,
//                                not a size-dependent duration)             (ns)
//   type 16 rccl_collective_ms   RCCL API call duration                      (ns)
//
// Timestamps are rocprofiler's monotonic clock, shifted to CLOCK_REALTIME once at init
// (the agent joins on wall-clock ns, like REF's decoder). Events below a per-signal floor
// are not emitted (the BPF probes apply the same kind of in-kernel filter),
// and a per-second budget caps the producer so a pathological workload cannot flood the
// ring (full rings drop, never block).
//
// Request tagging: a serving process calls mislo_rocprof_set_trace(hash) (C ABI, e.g. through
// ctypes on the already-loaded library) on the thread that runs a request; kernels that thread
// enqueues carry the hash (trace_h: the low 64 bits of the request's W3C trace id, the OTLP
// receiver's rule), so the agent joins them to the request's spans through the trace tier
// instead of the coarser pod+pid window.
//
// Environment: MISLO_RING (default /mislo-agent-events), MISLO_POD_ID, MISLO_NODE_ID,
// MISLO_SVC_ID, MISLO_HBM_BYTES (default 288 GiB), MISLO_MAX_EPS (default 200000),
// MISLO_QUEUE_FLOOR_NS (default 100000), MISLO_XGMI_GBPS (nominal peer-copy rate, default
// 64 GB/s: one xGMI link direction), MISLO_ROCPROF_VERBOSE.
#include <rocprofiler-sdk/buffer.h>
#include <rocprofiler-sdk/buffer_tracing.h>
#include <rocprofiler-sdk/callback_tracing.h>
#include <rocprofiler-sdk/fwd.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "mislo_record.h"

extern "C" {
void* mislo_ring_open_shm(const char* name);
uint32_t mislo_ring_rec_size(void* ring);
void mislo_ring_close(void* ring);
uint64_t mislo_ring_push_batch(void* ring, const void* recs, uint64_t n);
}

namespace {

struct alignas(64) EventRec {  // collector/records.py EVENT
  int64_t ts_ns;
  uint64_t value;
  uint64_t trace_h;
  uint32_t pid, tid, pod_id, dst_ip;
  uint16_t signal_type, node_id, svc_id, flags, src_port, dst_port;
  int32_t err;
  uint64_t conn_h;
};
static_assert(sizeof(EventRec) == 64, "EVENT layout");

struct User32Rec {  // collector/records.py USER32
  int64_t ts_ns;
  uint64_t trace_h;
  uint32_t value_milli, pod_id, pid;
  uint8_t signal_type, flags;
  uint16_t node_id;
};
static_assert(sizeof(User32Rec) == 32, "USER32 layout");

struct User24Rec {  // collector/records.py USER24 (ops/csrc/mislo_common.h User24)
  uint64_t trace_h;
  uint32_t value_milli, ts_lo;
  uint32_t pid_sig;  // pid | signal_type << 22 | ts_zero << 29 | has_gpu << 30
  uint32_t pod_ts;   // pod_id | (ts bits 32..43) << 20
};
static_assert(sizeof(User24Rec) == 24, "USER24 layout");

constexpr uint16_t kQueueDelay = 13, kHbmPressure = 14, kXgmiLatency = 15, kRcclCollective = 16;

struct State {
  rocprofiler_client_id_t* client = nullptr;
  rocprofiler_context_id_t ctx{};
  rocprofiler_buffer_id_t buffer{};
  void* ring = nullptr;
  int64_t clock_offset = 0;  // realtime - rocprofiler timestamp
  uint32_t pod = 0;
  uint16_t node = 0, svc = 0;
  uint64_t hbm_bytes = 288ull << 30;
  uint64_t max_eps = 200000;
  uint64_t queue_floor_ns = 100000;
  double xgmi_bytes_per_ns = 64.0;
  bool rec32 = false;  // the ring holds 32-byte USER32 records
  bool rec24 = false;  // the ring holds 24-byte USER24 records
  bool verbose = false;
  std::mutex mu;
  struct Enq {
    uint64_t ts, trace_h;
  };
  std::unordered_map<uint64_t, Enq> enqueue_ts;  // correlation id -> enqueue time, request trace
  std::unordered_map<uint64_t, uint64_t> live_alloc;  // address -> bytes
  uint64_t live_bytes = 0;
  uint64_t last_hbm_milli = ~0ull;
  std::atomic<uint64_t> window_sec{0}, window_count{0}, pushed{0}, dropped{0};
};

State g;
thread_local uint64_t t_trace = 0;  // the calling thread's current request (mislo_rocprof_set_trace)

uint64_t env_u64(const char* k, uint64_t d) {
  const char* v = std::getenv(k);
  return v && *v ? std::strtoull(v, nullptr, 0) : d;
}

uint32_t tid() { return (uint32_t)syscall(SYS_gettid); }

void emit(uint16_t type, uint64_t ts, uint64_t value, uint32_t thread, uint64_t trace_h = 0) {
  if (!g.ring) return;
  const int64_t wall = (int64_t)ts + g.clock_offset;
  const uint64_t sec = (uint64_t)wall / 1000000000ull;
  if (g.window_sec.load(std::memory_order_relaxed) != sec) {
    g.window_sec.store(sec, std::memory_order_relaxed);
    g.window_count.store(0, std::memory_order_relaxed);
  }
  if (g.window_count.fetch_add(1, std::memory_order_relaxed) >= g.max_eps) {
    g.dropped.fetch_add(1, std::memory_order_relaxed);
    return;
  }
  bool ok;
  if (g.rec24) {
    User24Rec u{};
    const uint64_t t = (uint64_t)wall;
    u.trace_h = trace_h;
    u.value_milli = mislo_milli(type, value);
    u.ts_lo = (uint32_t)t;
    u.pid_sig = ((uint32_t)getpid() & 0x3FFFFFu) | ((uint32_t)(type & 0x7F) << 22) | (wall == 0 ? 1u << 29 : 0u) |
                (1u << 30);
    u.pod_ts = (g.pod & 0xFFFFFu) | (uint32_t)(((t >> 32) & 0xFFFu) << 20);
    ok = mislo_ring_push_batch(g.ring, &u, 1) == 1;
    (ok ? g.pushed : g.dropped).fetch_add(1, std::memory_order_relaxed);
    return;
  }
  if (g.rec32) {
    User32Rec u{};
    u.ts_ns = wall;
    u.trace_h = trace_h;
    u.value_milli = mislo_milli(type, value);
    u.pod_id = g.pod;
    u.pid = (uint32_t)getpid();
    u.signal_type = (uint8_t)type;
    u.flags = 1;  // has_gpu
    u.node_id = g.node;
    ok = mislo_ring_push_batch(g.ring, &u, 1) == 1;
    (ok ? g.pushed : g.dropped).fetch_add(1, std::memory_order_relaxed);
    return;
  }
  EventRec e;
  std::memset(&e, 0, sizeof(e));
  e.ts_ns = wall;
  e.value = value;
  e.trace_h = trace_h;
  e.pid = (uint32_t)getpid();
  e.tid = thread ? thread : tid();
  e.pod_id = g.pod;
  e.node_id = g.node;
  e.svc_id = g.svc;
  e.signal_type = type;
  e.flags = 1u << 8;  // has_gpu
  if (mislo_ring_push_batch(g.ring, &e, 1) == 1)
    g.pushed.fetch_add(1, std::memory_order_relaxed);
  else
    g.dropped.fetch_add(1, std::memory_order_relaxed);
}

void emit_hbm(uint64_t ts) {
  // value in milli-percent of HBM capacity; emitted when it moves by >= 0.1 pct-point
  const uint64_t milli = g.hbm_bytes ? (uint64_t)((double)g.live_bytes * 100000.0 / (double)g.hbm_bytes) : 0;
  if (g.last_hbm_milli != ~0ull && (milli > g.last_hbm_milli ? milli - g.last_hbm_milli : g.last_hbm_milli - milli) < 100)
    return;
  g.last_hbm_milli = milli;
  emit(kHbmPressure, ts, milli, 0);
}

// Kernel dispatch ENQUEUE (host side) and COMPLETE (with device start/end timestamps).
void dispatch_callback(rocprofiler_callback_tracing_record_t rec, rocprofiler_user_data_t*, void*) {
  if (rec.kind != ROCPROFILER_CALLBACK_TRACING_KERNEL_DISPATCH) return;
  if (rec.operation == ROCPROFILER_KERNEL_DISPATCH_ENQUEUE && rec.phase == ROCPROFILER_CALLBACK_PHASE_ENTER) {
    rocprofiler_timestamp_t now = 0;
    rocprofiler_get_timestamp(&now);
    std::lock_guard<std::mutex> lk(g.mu);
    g.enqueue_ts[rec.correlation_id.internal] = State::Enq{now, t_trace};  // the enqueuing thread's request
  } else if (rec.operation == ROCPROFILER_KERNEL_DISPATCH_COMPLETE) {
    auto* d = static_cast<rocprofiler_callback_tracing_kernel_dispatch_data_t*>(rec.payload);
    State::Enq enq{0, 0};
    {
      std::lock_guard<std::mutex> lk(g.mu);
      auto it = g.enqueue_ts.find(rec.correlation_id.internal);
      if (it != g.enqueue_ts.end()) {
        enq = it->second;
        g.enqueue_ts.erase(it);
      }
    }
    if (enq.ts && d && d->start_timestamp > enq.ts) {
      const uint64_t delay = d->start_timestamp - enq.ts;
      if (delay >= g.queue_floor_ns)
        emit(kQueueDelay, d->start_timestamp, delay, (uint32_t)rec.thread_id, enq.trace_h);
    }
  }
}

void buffer_callback(rocprofiler_context_id_t, rocprofiler_buffer_id_t, rocprofiler_record_header_t** headers,
                     size_t n, void*, uint64_t) {
  for (size_t i = 0; i < n; ++i) {
    auto* h = headers[i];
    if (h->category != ROCPROFILER_BUFFER_CATEGORY_TRACING) continue;
    if (h->kind == ROCPROFILER_BUFFER_TRACING_MEMORY_COPY) {
      auto* r = static_cast<rocprofiler_buffer_tracing_memory_copy_record_t*>(h->payload);
      if (r->operation == ROCPROFILER_MEMORY_COPY_DEVICE_TO_DEVICE && r->src_agent_id.handle != r->dst_agent_id.handle &&
          r->end_timestamp > r->start_timestamp) {
        // latency = duration - bytes / nominal link rate: a healthy link moves a large copy
        // in ~its transfer time (latency ~ setup cost), a degraded or congested link does not
        const uint64_t dur = r->end_timestamp - r->start_timestamp;
        const uint64_t xfer = (uint64_t)((double)r->bytes / g.xgmi_bytes_per_ns);
        emit(kXgmiLatency, r->start_timestamp, dur > xfer ? dur - xfer : 0, (uint32_t)r->thread_id);
      }
    } else if (h->kind == ROCPROFILER_BUFFER_TRACING_MEMORY_ALLOCATION) {
      auto* r = static_cast<rocprofiler_buffer_tracing_memory_allocation_record_t*>(h->payload);
      std::lock_guard<std::mutex> lk(g.mu);
      const uint64_t addr = r->address.handle;
      if (r->operation == ROCPROFILER_MEMORY_ALLOCATION_ALLOCATE ||
          r->operation == ROCPROFILER_MEMORY_ALLOCATION_VMEM_ALLOCATE) {
        g.live_alloc[addr] = r->allocation_size;
        g.live_bytes += r->allocation_size;
      } else if (r->operation == ROCPROFILER_MEMORY_ALLOCATION_FREE ||
                 r->operation == ROCPROFILER_MEMORY_ALLOCATION_VMEM_FREE) {
        auto it = g.live_alloc.find(addr);
        if (it != g.live_alloc.end()) {
          g.live_bytes -= it->second;
          g.live_alloc.erase(it);
        }
      }
      emit_hbm(r->end_timestamp ? r->end_timestamp : r->start_timestamp);
    } else if (h->kind == ROCPROFILER_BUFFER_TRACING_RCCL_API) {
      auto* r = static_cast<rocprofiler_buffer_tracing_rccl_api_record_t*>(h->payload);
      if (r->end_timestamp > r->start_timestamp)
        emit(kRcclCollective, r->start_timestamp, r->end_timestamp - r->start_timestamp, (uint32_t)r->thread_id);
    }
  }
}

#define CHECK(x)                                                                          \
  do {                                                                                    \
    rocprofiler_status_t _s = (x);                                                        \
    if (_s != ROCPROFILER_STATUS_SUCCESS) {                                               \
      if (g.verbose) std::fprintf(stderr, "[mislo-rocprof] %s failed: %d\n", #x, (int)_s); \
      ok = false;                                                                         \
    }                                                                                     \
  } while (0)

int tool_init(rocprofiler_client_finalize_t, void*) {
  bool ok = true;
  const char* name = std::getenv("MISLO_RING");
  g.ring = mislo_ring_open_shm(name && *name ? name : "/mislo-agent-events");
  g.rec32 = g.ring && mislo_ring_rec_size(g.ring) == 32;
  g.rec24 = g.ring && mislo_ring_rec_size(g.ring) == 24;
  g.pod = (uint32_t)env_u64("MISLO_POD_ID", 0);
  g.node = (uint16_t)env_u64("MISLO_NODE_ID", 0);
  g.svc = (uint16_t)env_u64("MISLO_SVC_ID", 0);
  g.hbm_bytes = env_u64("MISLO_HBM_BYTES", 288ull << 30);
  g.max_eps = env_u64("MISLO_MAX_EPS", 200000);
  g.queue_floor_ns = env_u64("MISLO_QUEUE_FLOOR_NS", 100000);
  g.xgmi_bytes_per_ns = (double)env_u64("MISLO_XGMI_GBPS", 64);  // GB/s == bytes/ns
  g.verbose = env_u64("MISLO_ROCPROF_VERBOSE", 0) != 0;
  timespec rt{};
  clock_gettime(CLOCK_REALTIME, &rt);
  rocprofiler_timestamp_t now = 0;
  rocprofiler_get_timestamp(&now);
  g.clock_offset = ((int64_t)rt.tv_sec * 1000000000ll + rt.tv_nsec) - (int64_t)now;

  CHECK(rocprofiler_create_context(&g.ctx));
  rocprofiler_tracing_operation_t ops[] = {ROCPROFILER_KERNEL_DISPATCH_ENQUEUE, ROCPROFILER_KERNEL_DISPATCH_COMPLETE};
  CHECK(rocprofiler_configure_callback_tracing_service(g.ctx, ROCPROFILER_CALLBACK_TRACING_KERNEL_DISPATCH, ops, 2,
                                                       dispatch_callback, nullptr));
  constexpr size_t kBuf = 1 << 16;
  CHECK(rocprofiler_create_buffer(g.ctx, kBuf, kBuf - kBuf / 8, ROCPROFILER_BUFFER_POLICY_LOSSLESS, buffer_callback,
                                  nullptr, &g.buffer));
  CHECK(rocprofiler_configure_buffer_tracing_service(g.ctx, ROCPROFILER_BUFFER_TRACING_MEMORY_COPY, nullptr, 0,
                                                     g.buffer));
  CHECK(rocprofiler_configure_buffer_tracing_service(g.ctx, ROCPROFILER_BUFFER_TRACING_MEMORY_ALLOCATION, nullptr, 0,
                                                     g.buffer));
  {
    // RCCL tracing is only available when the workload links RCCL; not fatal if absent
    bool keep = ok;
    CHECK(rocprofiler_configure_buffer_tracing_service(g.ctx, ROCPROFILER_BUFFER_TRACING_RCCL_API, nullptr, 0,
                                                       g.buffer));
    ok = keep;
  }
  rocprofiler_callback_thread_t th{};
  CHECK(rocprofiler_create_callback_thread(&th));
  CHECK(rocprofiler_assign_callback_thread(g.buffer, th));
  int valid = 0;
  CHECK(rocprofiler_context_is_valid(g.ctx, &valid));
  if (!ok || !valid) return -1;
  CHECK(rocprofiler_start_context(g.ctx));
  if (g.verbose)
    std::fprintf(stderr, "[mislo-rocprof] started (ring=%s attached=%d)\n", name ? name : "/mislo-agent-events",
                 g.ring != nullptr);
  return ok ? 0 : -1;
}

void tool_fini(void*) {
  rocprofiler_flush_buffer(g.buffer);
  if (g.verbose)
    std::fprintf(stderr, "[mislo-rocprof] pushed=%llu dropped=%llu\n", (unsigned long long)g.pushed.load(),
                 (unsigned long long)g.dropped.load());
  if (g.ring) mislo_ring_close(g.ring);
  g.ring = nullptr;
}

}  // namespace

extern "C" {

// Counters for tests / the agent's ring statistics.
uint64_t mislo_rocprof_pushed() { return g.pushed.load(); }
uint64_t mislo_rocprof_dropped() { return g.dropped.load(); }

// The calling thread's current request trace (0 = none): kernels it enqueues from now on carry it.
void mislo_rocprof_set_trace(uint64_t trace_h) { t_trace = trace_h; }

rocprofiler_tool_configure_result_t* rocprofiler_configure(uint32_t, const char*, uint32_t,
                                                           rocprofiler_client_id_t* id) {
  id->name = "llm-slo-ebpf-toolkit-amd";
  g.client = id;
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init,
                                                 &tool_fini, nullptr};
  return &cfg;
}

}  // extern "C"
