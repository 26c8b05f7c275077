// rocprofiler-sdk tool library: the user-space GPU signal source of the MI355X agent.
//
// Loaded into an LLM workload (ROCP_TOOL_LIBRARIES=libmislo_rocprof.so, no root needed),
// it turns runtime activity into the four GPU signals of the catalogue and pushes them into
// the agent's shared-memory ring (runtime/csrc/ring.h C ABI) as the ring's record type: 64-byte
// EVENT or, in rings created with 32- or 24-byte records, USER32 / USER24 (collector/records.py;
// the value in fixed point by the probes' own rule, mislo_record.h mislo_milli; USER24 packs
// pid / type / pod id and keeps the timestamp's low 44 bits -- 3/8 of the PCIe bytes of EVENT):
//
//   type 13 gpu_queue_delay_ms   (a) kernel dispatch: start - max(enqueue return, queue predecessor end),
//                                when another process's waves were on the GPU during the wait (ns);
//                                (b) foreign GPU time: every MISLO_FOREIGN_MS (default 100) while this
//                                process runs kernels, the share of the interval other processes'
//                                waves held the GPU, as ns of the interval, when it reaches
//                                MISLO_FOREIGN_FLOOR_PCT (default 10). KFD reports each process's
//                                wave occupancy per GPU (/sys/class/kfd/kfd/proc/<pid>/stats_<gpu_id>/
//                                cu_occupancy, readable without root); every MISLO_OCC_MS (default
//                                10) at which this process has NO kernel in flight, the sum over all
//                                processes on its GPU is other processes' occupancy alone -- no need
//                                to know which host pid is this one (a container's pid namespace
//                                hides it), and immune to the inter-kernel overhead that made
//                                "device activity minus own kernel time" read 30 % busy for a
//                                decode loop of microsecond kernels alone on the GPU (r4 box).
//                                Meanwhile the tool learns its own entry (never holding waves at
//                                those idle readings, most often while it has kernels in flight);
//                                from then on every reading counts, minus its own entry -- a
//                                saturated server has no idle moments at all (ns)
//   type 14 hbm_pressure_pct     the GPU's node-wide HBM use: amdgpu sysfs mem_info_vram_used /
//                                mem_info_vram_total of the PCI device the process allocates on
//                                (every process's allocations, not this one's), sampled on
//                                allocations and every MISLO_HBM_SAMPLE_MS (milli-pct)
//   type 15 xgmi_link_latency_us peer GPU copy latency, calibrated per (src, dst) GPU pair: a
//                                small copy (<= 64 KiB) is all latency; a larger one's latency is
//                                its time beyond its bytes at the best rate that pair has shown
//                                (its calibrated bandwidth, large copies only)             (ns)
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
// Split rings (agent --gpus N): MISLO_RING may list one ring per window worker ("a,b,..."); the
// records go to the ring of the worker that owns this process's pod, read from the agent's
// shared-memory pod -> shard table (MISLO_SHARD_TABLE, one byte per pod id; re-read every sample
// tick, so a pod the agent routes later follows). Without a table, the first ring.
//
// Shedding: the agent's overhead guard sets bits in the ring header's drop mask (runtime/csrc/ring.h);
// a record whose signal type's bit is set is not emitted (counted as dropped).
//
// Environment: MISLO_RING (default /mislo-agent-events), MISLO_POD_ID, MISLO_NODE_ID,
// MISLO_SVC_ID, MISLO_HBM_BYTES (fallback capacity when sysfs is unreadable, default 288 GiB),
// MISLO_PCI_SYSFS (default /sys/bus/pci/devices), MISLO_HBM_SAMPLE_MS (default 1000),
// MISLO_MAX_EPS (default 200000), MISLO_QUEUE_FLOOR_NS (default 10 ms: below that a dispatch's wait
// on an otherwise idle GPU is clock / power-state ramp, not another process -- config-2 baselines
// read 2-5 ms waits there, while contention shows up as foreign GPU time), MISLO_XGMI_GBPS (a
// pair's starting rate before it has shown a large copy, default 64 GB/s: one xGMI link
// direction; a pair's calibration starts there and a measured rate may only raise it, to at most
// 4x: a link already degraded when the process starts is not its own baseline),
// MISLO_FOREIGN_MS, MISLO_FOREIGN_FLOOR_PCT, MISLO_FOREIGN_MIN_HOT (default 2 readings with foreign waves
// per interval), MISLO_OCC_MS, MISLO_FOREIGN_MIN_SAMPLES (default 3 idle
// samples per interval), MISLO_KFD_PROC (default /sys/class/kfd/kfd/proc), MISLO_WAIT_NEEDS_FOREIGN
// (default 1: where KFD's process directory exists, a dispatch wait is emitted only if a reading
// saw another process hold waves on the GPU during it, none before the first reading -- a
// CPU-starved process's kernels wait behind its own host-staged copies and barriers too; 0 =
// every wait above the floor), MISLO_ROCPROF_VERBOSE.
#include <rocprofiler-sdk/buffer.h>
#include <rocprofiler-sdk/buffer_tracing.h>
#include <rocprofiler-sdk/callback_tracing.h>
#include <rocprofiler-sdk/fwd.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <vector>
#include <chrono>
#include <condition_variable>
#include <map>
#include <string>
#include <thread>
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
uint32_t mislo_ring_drop_mask(void* ring);
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
  // the ring records go to now (rings[shard]): route() switches it on the sampler thread while the
  // callback threads emit, so each emit() loads it once and uses that ring for both the drop-mask
  // check and the push
  std::atomic<void*> ring{nullptr};
  std::vector<void*> rings;            // MISLO_RING's rings, one per window worker
  const uint8_t* shard_table = nullptr;  // pod id -> shard (MISLO_SHARD_TABLE), 2^20 bytes
  int64_t clock_offset = 0;  // realtime - rocprofiler timestamp
  uint32_t pod = 0;
  uint16_t node = 0, svc = 0;
  uint64_t hbm_bytes = 288ull << 30;
  uint64_t max_eps = 200000;
  uint64_t queue_floor_ns = 10000000;
  double xgmi_bytes_per_ns = 64.0;
  bool rec32 = false;  // the ring holds 32-byte USER32 records
  bool rec24 = false;  // the ring holds 24-byte USER24 records
  bool rec16 = false;  // the ring holds 16-byte USER16 slots (a traced record takes two)
  bool verbose = false;
  std::mutex mu;
  struct Enq {
    uint64_t ts, trace_h, pred;  // pred: dispatch id of the same queue's previous dispatch (0: none)
  };
  std::unordered_map<uint64_t, Enq> enqueue_ts;  // correlation id -> enqueue time, request trace
  std::unordered_map<uint64_t, uint64_t> queue_last;  // HW queue -> its latest enqueued dispatch id
  std::unordered_map<uint64_t, uint64_t> disp_end;    // dispatch id -> end, until its successor completes
  std::unordered_map<uint64_t, uint64_t> live_alloc;  // address -> bytes
  uint64_t live_bytes = 0;
  // node-wide HBM of the GPUs this process uses: agent handle -> the PCI device's VRAM counters
  struct Vram {
    int used_fd = -1, total_fd = -1;
    uint64_t last_milli = ~0ull;
  };
  std::map<uint64_t, Vram> vram;
  std::mutex hbm_mu;  // emit_hbm runs on the sampler thread and the buffer callback thread
  // foreign GPU time per GPU agent (KFD gpu_id): this process's kernels in flight (enqueued, not
  // yet completed; guarded by mu) gate the sampler thread's occupancy readings
  struct Occ {
    uint64_t gpu_id = 0;
    int64_t inflight = 0;          // mu
    uint64_t enq_seq = 0;          // mu: enqueues so far (a reading that straddles one is dropped)
    uint64_t disp = 0;             // mu: enqueues in the current interval
    uint64_t last_read = 0;        // sampler thread: time of the last reading (ns)
    uint64_t last_done = 0;        // mu: last completion, or the enqueue that ended an idle spell (ns)
    // sampler thread only: the current interval's idle readings
    uint64_t t0 = 0, t_first = 0, clean = 0, hot = 0, busy_skips = 0;
    double occ_sum = 0.0;
    // last decided interval and the reading cost (tests, overhead accounting)
    double share = 0.0, occ_mean = 0.0;
    uint64_t decisions = 0, reads = 0, read_ns = 0, cleans = 0, emitted = 0;
    // mu: the latest counted reading with other processes' waves on the GPU (ns; 0 = never) and
    // whether readings work at all -- a dispatch wait counts as contention only when foreign waves
    // were seen during it (a host-starved process's kernels also wait, behind its own staged
    // copies and host-signalled barriers: profiles/r4_config3 read that as gpu_contention)
    uint64_t last_foreign = 0;
    bool readable = false;
    uint64_t waits_emitted = 0, waits_unconfirmed = 0;
    // which KFD entry is this process (a container's pid namespace hides its host pid): the entry
    // that never holds waves while this process has none in flight, and most often does while it
    // has -- learned from the readings; once known, every reading counts, in flight or not
    struct Cand {
      uint64_t idle_hot = 0, busy_hot = 0;
    };
    std::map<uint32_t, Cand> cands;
    uint64_t idle_n = 0, busy_n = 0;
    uint32_t self_pid = 0;  // 0: not identified yet
  };
  std::map<uint64_t, Occ> occ;
  uint64_t foreign_ms = 100, foreign_floor_pct = 10, occ_ms = 10, foreign_min_samples = 3, foreign_min_hot = 2;
  bool wait_needs_foreign = true;
  bool kfd_dir = false;  // the KFD process directory is there: occupancy can confirm waits
  std::string kfd_proc = "/sys/class/kfd/kfd/proc";
  std::string pci_sysfs = "/sys/bus/pci/devices";
  uint64_t hbm_sample_ms = 1000;
  uint64_t last_hbm_milli = ~0ull;  // fallback (no sysfs): this process's live allocations
  // per (src, dst) agent pair: calibrated bandwidth (bytes/ns, best large copy) and the smallest
  // small-copy latency seen
  struct Link {
    double bytes_per_ns = 0.0;
    uint64_t min_small_ns = ~0ull;
    uint64_t copies = 0;
  };
  std::map<std::pair<uint64_t, uint64_t>, Link> links;
  std::thread sampler;
  std::mutex smu;
  std::condition_variable scv;
  bool stop = false;
  std::atomic<bool> kick{false};  // a GPU went idle for this process: take an occupancy reading now
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
  void* const ring = g.ring.load(std::memory_order_acquire);
  if (!ring) return;
  if (type < 32 && (mislo_ring_drop_mask(ring) >> type & 1u)) {  // shed by the agent's overhead guard
    g.dropped.fetch_add(1, std::memory_order_relaxed);
    return;
  }
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
  if (g.rec16) {  // collector/records.py USER16: {ts_lo, value, pid_sig, pod_ts} [+ {trace, marker, 0}]
    const uint64_t t = (uint64_t)wall;
    uint32_t w[8] = {};
    w[0] = (uint32_t)t;
    w[1] = mislo_milli(type, value);
    w[2] = ((uint32_t)getpid() & 0x3FFFFFu) | ((uint32_t)(type & 0x7F) << 22) | (wall == 0 ? 1u << 29 : 0u) |
           (1u << 30) | (trace_h ? 1u << 31 : 0u);
    w[3] = (g.pod & 0xFFFFFu) | (uint32_t)(((t >> 32) & 0xFFFu) << 20);
    w[4] = (uint32_t)trace_h;
    w[5] = (uint32_t)(trace_h >> 32);
    w[6] = 0xFFFFFFFFu;  // continuation marker
    const uint64_t n = trace_h ? 2 : 1;  // one batch: a window never splits a record from its trace
    ok = mislo_ring_push_batch(ring, w, n) == n;
    (ok ? g.pushed : g.dropped).fetch_add(1, std::memory_order_relaxed);
    return;
  }
  if (g.rec24) {
    User24Rec u{};
    const uint64_t t = (uint64_t)wall;
    u.trace_h = trace_h;
    u.value_milli = mislo_milli(type, value);
    u.ts_lo = (uint32_t)t;
    u.pid_sig = ((uint32_t)getpid() & 0x3FFFFFu) | ((uint32_t)(type & 0x7F) << 22) | (wall == 0 ? 1u << 29 : 0u) |
                (1u << 30);
    u.pod_ts = (g.pod & 0xFFFFFu) | (uint32_t)(((t >> 32) & 0xFFFu) << 20);
    ok = mislo_ring_push_batch(ring, &u, 1) == 1;
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
    ok = mislo_ring_push_batch(ring, &u, 1) == 1;
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
  if (mislo_ring_push_batch(ring, &e, 1) == 1)
    g.pushed.fetch_add(1, std::memory_order_relaxed);
  else
    g.dropped.fetch_add(1, std::memory_order_relaxed);
}

uint64_t read_u64_fd(int fd) {
  char buf[32];
  const ssize_t n = pread(fd, buf, sizeof(buf) - 1, 0);
  if (n <= 0) return 0;
  buf[n] = 0;
  return std::strtoull(buf, nullptr, 10);
}

// HBM pressure of one GPU in milli-percent: node-wide VRAM use from the amdgpu driver (every
// process on the GPU), or -- without sysfs -- this process's live allocations over the capacity.
bool hbm_milli(uint64_t agent, uint64_t* out, uint64_t** last) {
  auto it = g.vram.find(agent);
  if (it != g.vram.end() && it->second.used_fd >= 0 && it->second.total_fd >= 0) {
    const uint64_t used = read_u64_fd(it->second.used_fd), total = read_u64_fd(it->second.total_fd);
    if (total) {
      *out = (uint64_t)((double)used * 100000.0 / (double)total);
      *last = &it->second.last_milli;
      return true;
    }
  }
  *out = g.hbm_bytes ? (uint64_t)((double)g.live_bytes * 100000.0 / (double)g.hbm_bytes) : 0;
  *last = &g.last_hbm_milli;
  return true;
}

// emitted when the GPU's pressure moved by >= 0.1 pct-point since its last record
void emit_hbm(uint64_t ts, uint64_t agent) {
  std::lock_guard<std::mutex> lk(g.hbm_mu);
  uint64_t milli = 0, *last = nullptr;
  if (!hbm_milli(agent, &milli, &last)) return;
  if (*last != ~0ull && (milli > *last ? milli - *last : *last - milli) < 100) return;
  *last = milli;
  emit(kHbmPressure, ts, milli, 0);
}

// A peer copy's xGMI latency on its (src, dst) pair, calibrating the pair as it goes.
uint64_t xgmi_latency(uint64_t src, uint64_t dst, uint64_t bytes, uint64_t dur) {
  std::lock_guard<std::mutex> lk(g.mu);
  State::Link& l = g.links[{src, dst}];
  if (l.copies == 0) l.bytes_per_ns = g.xgmi_bytes_per_ns;  // nominal: a measured rate only raises it
  ++l.copies;
  if (bytes <= (64u << 10)) {  // small copy: the duration is the link's latency
    if (dur < l.min_small_ns) l.min_small_ns = dur;
    return dur;
  }
  const double rate = (double)bytes / (double)dur;
  if (bytes >= (1u << 20) && rate > l.bytes_per_ns)  // calibrated bandwidth, at most 4x the nominal rate
    l.bytes_per_ns = rate < 4.0 * g.xgmi_bytes_per_ns ? rate : 4.0 * g.xgmi_bytes_per_ns;
  const double bw = l.bytes_per_ns > 0.0 ? l.bytes_per_ns : g.xgmi_bytes_per_ns;
  const uint64_t xfer = (uint64_t)((double)bytes / bw);
  return dur > xfer ? dur - xfer : 0;
}

// Every KFD process's cu_occupancy on one GPU (CU-equivalents of resident waves): (host pid,
// occupancy) of the processes with a stats_<gpu_id> directory -- the others are not on this GPU.
// The files stay open between readings (one pread each); the process tree is re-listed every
// 500 ms for processes that came and went -- an opendir plus an open / read / close per process
// cost ~130 us a reading (profiles/r4_config3_gated/rocprof_tool.log, read_us).
struct OccFiles {
  std::vector<std::pair<uint32_t, int>> fds;  // (host pid, cu_occupancy fd)
  std::chrono::steady_clock::time_point listed{};
  bool have = false;
};

void occ_list(uint64_t gpu_id, OccFiles& f) {
  std::map<uint32_t, int> old;
  for (const auto& e : f.fds) old[e.first] = e.second;
  std::vector<std::pair<uint32_t, int>> next;
  if (DIR* d = opendir(g.kfd_proc.c_str())) {
    char path[512];
    while (dirent* e = readdir(d)) {
      if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
      const uint32_t pid = (uint32_t)std::strtoul(e->d_name, nullptr, 10);
      const auto it = old.find(pid);
      if (it != old.end()) {
        next.emplace_back(pid, it->second);
        old.erase(it);
        continue;
      }
      std::snprintf(path, sizeof(path), "%s/%s/stats_%llu/cu_occupancy", g.kfd_proc.c_str(), e->d_name,
                    (unsigned long long)gpu_id);
      const int fd = open(path, O_RDONLY | O_CLOEXEC);
      if (fd >= 0) next.emplace_back(pid, fd);
    }
    closedir(d);
  }
  for (const auto& kv : old) close(kv.second);
  f.fds.swap(next);
  f.listed = std::chrono::steady_clock::now();
  f.have = true;
}

bool kfd_occupancy(uint64_t gpu_id, std::vector<std::pair<uint32_t, uint64_t>>* out) {
  static std::mutex mu;  // the sampler thread, and init's readability check
  static std::map<uint64_t, OccFiles> files;
  std::lock_guard<std::mutex> lk(mu);
  out->clear();
  OccFiles& f = files[gpu_id];
  if (!f.have || std::chrono::steady_clock::now() - f.listed > std::chrono::milliseconds(500)) occ_list(gpu_id, f);
  char buf[32];
  for (size_t i = 0; i < f.fds.size();) {
    const ssize_t n = pread(f.fds[i].second, buf, sizeof(buf) - 1, 0);
    if (n <= 0) {  // the process is gone
      close(f.fds[i].second);
      f.fds.erase(f.fds.begin() + (std::ptrdiff_t)i);
      continue;
    }
    buf[n] = 0;
    out->emplace_back(f.fds[i].first, std::strtoull(buf, nullptr, 10));
    ++i;
  }
  return !out->empty();
}

// Which entry is this process: never hot at its idle readings (<= 1 %), hot at the most of its
// busy ones, clearly ahead of the runner-up. Re-checked as readings accrue; a choice that starts
// holding waves while this process is idle is dropped.
void identify_self(State::Occ& o) {
  if (o.self_pid) {
    const auto it = o.cands.find(o.self_pid);
    if (it == o.cands.end() || (o.idle_n >= 100 && it->second.idle_hot * 100 > o.idle_n)) o.self_pid = 0;
    return;
  }
  if (o.idle_n < 20 || o.busy_n < 20) return;
  uint32_t best = 0;
  uint64_t b1 = 0, b2 = 0;
  for (const auto& kv : o.cands) {
    if (kv.second.idle_hot * 100 > o.idle_n) continue;
    if (kv.second.busy_hot > b1) {
      b2 = b1, b1 = kv.second.busy_hot, best = kv.first;
    } else if (kv.second.busy_hot > b2) {
      b2 = kv.second.busy_hot;
    }
  }
  if (best && b1 >= 5 && 2 * b2 < b1) o.self_pid = best;
}

// One occupancy reading per GPU this process is using. Idle (no kernel of this process in flight,
// none enqueued during the reading): every entry's waves are other processes' -- and a lesson for
// identify_self. In flight: only once this process's own entry is known, other entries' waves.
void occ_sample(uint64_t now) {
  static thread_local std::vector<std::pair<uint32_t, uint64_t>> per;
  for (auto& kv : g.occ) {
    State::Occ& o = kv.second;
    if (!o.gpu_id) continue;
    uint64_t seq = 0;
    bool idle = false, active = false;
    {
      std::lock_guard<std::mutex> lk(g.mu);
      // in flight with no completion for 5 s: a lost completion, not a kernel still running
      if (o.inflight > 0 && now > o.last_done + 5000000000ull) o.inflight = 0;
      idle = o.inflight <= 0;
      // serving: it enqueued in this interval, or kernels of it are still queued / running (a
      // contended prefill enqueues in a burst, then waits on them for most of a second)
      active = o.disp > 0 || !idle;
      if (!idle) o.disp += o.disp == 0;  // the interval counts as one this process used the GPU in
      seq = o.enq_seq;
    }
    if (!active) continue;  // not serving: no readings
    // at most two readings per MISLO_OCC_MS (a reading costs ~70 us of this thread on the r4 box)
    if (now < o.last_read + g.occ_ms * 500000ull) continue;
    o.last_read = now;
    const auto t = std::chrono::steady_clock::now();
    const bool ok = kfd_occupancy(o.gpu_id, &per);
    o.read_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t).count();
    ++o.reads;
    if (!ok) continue;
    bool busy = false;
    {
      std::lock_guard<std::mutex> lk(g.mu);
      const bool still_idle = o.inflight <= 0 && o.enq_seq == seq;
      busy = !idle && o.inflight > 0;
      if (idle && !still_idle) continue;  // this process enqueued meanwhile: neither kind
    }
    if (!idle && !busy) continue;
    uint64_t total = 0, self = 0;
    for (const auto& e : per) {
      total += e.second;
      if (e.first == o.self_pid) self = e.second;
      if (e.second) {
        State::Occ::Cand& c = o.cands[e.first];
        ++(idle ? c.idle_hot : c.busy_hot);
      } else {
        o.cands.emplace(e.first, State::Occ::Cand{});
      }
    }
    ++(idle ? o.idle_n : o.busy_n);
    if (o.cands.size() > 4096) o.cands.clear(), o.idle_n = o.busy_n = 0, o.self_pid = 0;  // pid churn
    if ((o.idle_n + o.busy_n) % 16 == 0) identify_self(o);
    if (busy && !o.self_pid) {
      ++o.busy_skips;
      continue;
    }
    const uint64_t foreign = total - (idle ? 0 : self);
    {
      std::lock_guard<std::mutex> lk(g.mu);
      o.readable = true;
      if (foreign > 0) o.last_foreign = now;
    }
    if (!o.clean) o.t_first = now;
    ++o.clean, ++o.cleans;
    o.occ_sum += (double)foreign;
    if (foreign > 0) ++o.hot;
  }
}

// Every foreign_ms, per GPU this process ran kernels on in the interval: the share of its idle
// readings at which other processes held waves on the GPU, emitted as that share of the interval.
// A busy process has few idle moments (a contended decode loop: ~1 per step): an interval with
// fewer than foreign_min_samples readings is extended, up to 10 x foreign_ms, before it is decided.
void foreign_tick(uint64_t now) {
  for (auto& kv : g.occ) {
    State::Occ& o = kv.second;
    if (o.t0 && o.clean < g.foreign_min_samples && now < o.t0 + 10 * g.foreign_ms * 1000000ull) continue;
    uint64_t disp = 0;
    {
      std::lock_guard<std::mutex> lk(g.mu);
      disp = o.disp;
      o.disp = 0;
    }
    // the interval starts at its first reading (less one reading period): a stretch without any
    // (the process idle, not serving) is not reported with the share seen after it
    const uint64_t t0 = o.t0 && o.t_first ? std::max(o.t0, o.t_first - std::min<uint64_t>(o.t_first, g.occ_ms * 1000000ull)) : o.t0;
    const uint64_t clean = o.clean, hot = o.hot;
    const double occ_sum = o.occ_sum;
    o.t0 = now, o.t_first = 0, o.clean = 0, o.hot = 0, o.occ_sum = 0.0;
    if (!t0 || now <= t0 || !disp || clean < g.foreign_min_samples) continue;
    const uint64_t dt = now - t0;
    o.share = (double)hot / (double)clean;
    o.occ_mean = occ_sum / (double)clean;
    ++o.decisions;
    // one hot reading is not evidence: a process alone on the GPU reads a few of its own waves as
    // another's when they race its idle check (2 such intervals in ~60 of the foreign test's alone phase)
    if (hot >= g.foreign_min_hot && o.share * 100.0 >= (double)g.foreign_floor_pct) {
      // an extended interval is reported as foreign_ms pieces, so the records keep the time
      // resolution the agent's join tiers need (pod + pid: 100 ms of the request span)
      const uint64_t step = g.foreign_ms * 1000000ull;
      const uint64_t k = std::max<uint64_t>(1, (dt + step / 2) / step);
      for (uint64_t j = 0; j < k; ++j) {
        const uint64_t a = t0 + dt * j / k, b = t0 + dt * (j + 1) / k;
        emit(kQueueDelay, a + (b - a) / 2, (uint64_t)(o.share * (double)(b - a)), 0);
      }
      ++o.emitted;
    }
  }
}

// Follow the agent's routing of this process's pod (split rings).
void route() {
  if (!g.shard_table || g.rings.size() < 2) return;
  const uint8_t s = g.shard_table[g.pod & 0xFFFFFu];
  void* r = g.rings[s < g.rings.size() ? s : 0];
  if (r) g.ring.store(r, std::memory_order_release);
}

void sampler_main() {
  std::unique_lock<std::mutex> lk(g.smu);
  const uint64_t tick = g.foreign_ms ? (g.hbm_sample_ms ? std::min(g.occ_ms, g.hbm_sample_ms) : g.occ_ms)
                                     : g.hbm_sample_ms;
  uint64_t next_hbm = 0, next_foreign = 0, next_tick = 0, next_report = 0;
  for (;;) {
    g.scv.wait_for(lk, std::chrono::milliseconds(tick), [] { return g.stop || g.kick.load(); });
    if (g.stop) break;
    rocprofiler_timestamp_t now = 0;
    rocprofiler_get_timestamp(&now);
    if (g.kick.exchange(false) && now < next_tick) {  // woken by an idle GPU between ticks
      occ_sample(now);
      continue;
    }
    next_tick = now + tick * 1000000ull - 500000ull;
    route();
    if (g.hbm_sample_ms && now >= next_hbm) {
      next_hbm = now + g.hbm_sample_ms * 1000000ull - 500000ull;
      for (auto& kv : g.vram)
        if (kv.second.last_milli != ~0ull) emit_hbm(now, kv.first);  // the GPUs this process has used
    }
    if (g.foreign_ms) {
      occ_sample(now);
      if (now >= next_foreign) {
        next_foreign = now + g.foreign_ms * 1000000ull - 500000ull;
        foreign_tick(now);
      }
      if (g.verbose && now >= next_report) {
        next_report = now + 10000000000ull;
        for (auto& kv : g.occ) {
          int64_t inflight = 0;
          uint64_t w_ok = 0, w_no = 0;
          {
            std::lock_guard<std::mutex> lk2(g.mu);
            inflight = kv.second.inflight;
            w_ok = kv.second.waits_emitted, w_no = kv.second.waits_unconfirmed;
          }
          std::fprintf(stderr,
                       "[mislo-rocprof] occupancy gpu_id %llu: dispatch waits emitted=%llu unconfirmed=%llu\n",
                       (unsigned long long)kv.second.gpu_id, (unsigned long long)w_ok, (unsigned long long)w_no);
          std::fprintf(stderr,
                       "[mislo-rocprof] occupancy gpu_id %llu: reads=%llu counted=%llu busy_skips=%llu decisions=%llu "
                       "emitted=%llu last_share=%.3f inflight=%lld read_us=%.1f self=%u (idle %llu busy %llu)\n",
                       (unsigned long long)kv.second.gpu_id, (unsigned long long)kv.second.reads,
                       (unsigned long long)kv.second.cleans, (unsigned long long)kv.second.busy_skips,
                       (unsigned long long)kv.second.decisions, (unsigned long long)kv.second.emitted, kv.second.share,
                       (long long)inflight, kv.second.reads ? kv.second.read_ns / 1e3 / kv.second.reads : 0.0,
                       kv.second.self_pid, (unsigned long long)kv.second.idle_n, (unsigned long long)kv.second.busy_n);
        }
      }
    }
  }
}

rocprofiler_status_t agents_cb(rocprofiler_agent_version_t, const void** agents, size_t n, void*) {
  for (size_t i = 0; i < n; ++i) {
    const auto* a = static_cast<const rocprofiler_agent_v0_t*>(agents[i]);
    if (a->type != ROCPROFILER_AGENT_TYPE_GPU) continue;
    char bdf[32];
    std::snprintf(bdf, sizeof(bdf), "%04x:%02x:%02x.%x", a->domain & 0xFFFF, (a->location_id >> 8) & 0xFF,
                  (a->location_id >> 3) & 0x1F, a->location_id & 7);
    State::Vram v;
    v.used_fd = open((g.pci_sysfs + "/" + bdf + "/mem_info_vram_used").c_str(), O_RDONLY | O_CLOEXEC);
    v.total_fd = open((g.pci_sysfs + "/" + bdf + "/mem_info_vram_total").c_str(), O_RDONLY | O_CLOEXEC);
    if (g.verbose)
      std::fprintf(stderr, "[mislo-rocprof] GPU %s: vram sysfs %s\n", bdf, v.used_fd >= 0 ? "ok" : "unreadable");
    g.vram[a->id.handle] = v;
    State::Occ& o = g.occ[a->id.handle];
    o.gpu_id = a->gpu_id;
    if (g.verbose) {
      std::vector<std::pair<uint32_t, uint64_t>> per;
      std::fprintf(stderr, "[mislo-rocprof] GPU %s: kfd gpu_id %llu occupancy %s\n", bdf, (unsigned long long)a->gpu_id,
                   kfd_occupancy(a->gpu_id, &per) ? "readable" : "unreadable (no foreign-time signal)");
    }
  }
  return ROCPROFILER_STATUS_SUCCESS;
}

// Kernel dispatch ENQUEUE (host side) and COMPLETE (with device start/end timestamps).
// gpu_queue_delay is the time a dispatch that COULD run waited for the device:
//   start - max(enqueue return, end of the previous dispatch on the same HW queue).
// * The enqueue time is taken when the enqueue returns (packet written, doorbell rung): from its
//   entry, a launching thread preempted inside the enqueue counted as GPU delay.
// * Waiting behind the process's own earlier dispatches on an in-order queue is not contention:
//   a CPU-starved launcher enqueues in bursts, and each kernel of a burst then queues behind the
//   previous one (config-3 run: 700-900 "warning" queue delays per phase while only the CPUs
//   were contended). What remains is the wait for compute units other work holds.
// The predecessor is the dispatch enqueued on the same queue just before (recorded at enqueue), not
// the latest completion seen: completion callbacks can arrive out of order, and a later
// dispatch's end taken for an earlier one's predecessor made the whole self-queued burst read as
// delay (a one-stream GEMM burst: 27 records up to 19 ms on one box). When the predecessor's
// completion has not been delivered yet, the dispatch emits nothing: on an in-order queue it
// started after that end, at an unknown point, so the wait behind its own queue is not separable.
void dispatch_callback(rocprofiler_callback_tracing_record_t rec, rocprofiler_user_data_t*, void*) {
  if (rec.kind != ROCPROFILER_CALLBACK_TRACING_KERNEL_DISPATCH) return;
  auto* d = static_cast<rocprofiler_callback_tracing_kernel_dispatch_data_t*>(rec.payload);
  if (rec.operation == ROCPROFILER_KERNEL_DISPATCH_ENQUEUE && rec.phase == ROCPROFILER_CALLBACK_PHASE_ENTER && d) {
    // in flight from before the packet is submitted: its completion can only come after this
    // (counted at the enqueue's exit, a fast kernel's completion could overtake the count)
    rocprofiler_timestamp_t now = 0;
    rocprofiler_get_timestamp(&now);
    std::lock_guard<std::mutex> lk(g.mu);
    auto oi = g.occ.find(d->dispatch_info.agent_id.handle);
    if (oi != g.occ.end()) {
      if (oi->second.inflight++ <= 0) oi->second.last_done = now;
      ++oi->second.enq_seq, ++oi->second.disp;
    }
  } else if (rec.operation == ROCPROFILER_KERNEL_DISPATCH_ENQUEUE && rec.phase == ROCPROFILER_CALLBACK_PHASE_EXIT) {
    rocprofiler_timestamp_t now = 0;
    rocprofiler_get_timestamp(&now);
    std::lock_guard<std::mutex> lk(g.mu);
    uint64_t pred = 0;
    if (d) {
      uint64_t& last = g.queue_last[d->dispatch_info.queue_id.handle];
      pred = last;
      last = d->dispatch_info.dispatch_id;
    }
    g.enqueue_ts[rec.correlation_id.internal] = State::Enq{now, t_trace, pred};  // the enqueuing thread's request
  } else if (rec.operation == ROCPROFILER_KERNEL_DISPATCH_COMPLETE) {
    State::Enq enq{0, 0, 0};
    {
      std::lock_guard<std::mutex> lk(g.mu);
      auto it = g.enqueue_ts.find(rec.correlation_id.internal);
      if (it != g.enqueue_ts.end()) {
        enq = it->second;
        g.enqueue_ts.erase(it);
      }
      if (d) {  // no longer in flight
        auto oi = g.occ.find(d->dispatch_info.agent_id.handle);
        if (oi != g.occ.end()) {
          if (oi->second.inflight > 0 && --oi->second.inflight == 0 && g.foreign_ms) {
            g.kick.store(true);  // idle now: the sampler reads other processes' occupancy
            g.scv.notify_one();
          }
          rocprofiler_timestamp_t now = 0;
          rocprofiler_get_timestamp(&now);
          oi->second.last_done = now;
        }
      }
    }
    if (!d) return;
    uint64_t ready = enq.ts;
    bool known = true;
    uint64_t last_foreign = 0;
    bool gated = false;
    State::Occ* occ = nullptr;
    {
      std::lock_guard<std::mutex> lk(g.mu);
      auto oi = g.occ.find(d->dispatch_info.agent_id.handle);
      // gated as soon as KFD's process directory exists, before the first reading: a wait with no
      // reading of foreign waves behind it is not emitted (a CPU-starved process's sampler thread
      // may not have read once yet -- it shares the starved CPU)
      if (oi != g.occ.end() && g.foreign_ms && g.wait_needs_foreign && (oi->second.readable || g.kfd_dir)) {
        occ = &oi->second;
        gated = true;
        last_foreign = occ->last_foreign;
      }
      if (g.disp_end.size() > 65536) g.disp_end.clear();  // ends whose successor never completed
      g.disp_end[d->dispatch_info.dispatch_id] = d->end_timestamp;
      if (enq.pred) {
        auto pe = g.disp_end.find(enq.pred);
        if (pe == g.disp_end.end()) {
          known = false;
        } else {
          if (pe->second > ready) ready = pe->second;
          g.disp_end.erase(pe);  // its successor is done with it
        }
      }
    }
    if (known && enq.ts && d->start_timestamp > ready) {
      const uint64_t delay = d->start_timestamp - ready;
      // with occupancy readable: only a wait during which another process held waves (one
      // reading period of slack: readings are MISLO_OCC_MS apart)
      const bool confirmed = !gated || last_foreign + g.occ_ms * 1000000ull >= ready;
      if (delay >= g.queue_floor_ns) {
        if (confirmed)
          emit(kQueueDelay, d->start_timestamp, delay, (uint32_t)rec.thread_id, enq.trace_h);
        std::lock_guard<std::mutex> lk(g.mu);
        if (occ) ++(confirmed ? occ->waits_emitted : occ->waits_unconfirmed);
      }
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
        // a healthy link moves a copy in its latency plus its bytes at the pair's calibrated
        // rate; a degraded or congested link does not
        const uint64_t dur = r->end_timestamp - r->start_timestamp;
        emit(kXgmiLatency, r->start_timestamp, xgmi_latency(r->src_agent_id.handle, r->dst_agent_id.handle, r->bytes, dur),
             (uint32_t)r->thread_id);
      }
    } else if (h->kind == ROCPROFILER_BUFFER_TRACING_MEMORY_ALLOCATION) {
      auto* r = static_cast<rocprofiler_buffer_tracing_memory_allocation_record_t*>(h->payload);
      std::unique_lock<std::mutex> lk(g.mu);
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
      lk.unlock();
      emit_hbm(r->end_timestamp ? r->end_timestamp : r->start_timestamp, r->agent_id.handle);
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
  {
    const std::string list = name && *name ? name : "/mislo-agent-events";
    size_t a = 0;
    while (a <= list.size()) {
      size_t b = list.find(',', a);
      if (b == std::string::npos) b = list.size();
      if (b > a) g.rings.push_back(mislo_ring_open_shm(list.substr(a, b - a).c_str()));
      a = b + 1;
    }
    g.ring.store(g.rings.empty() ? nullptr : g.rings[0], std::memory_order_release);
    if (const char* t = std::getenv("MISLO_SHARD_TABLE")) {
      const int fd = shm_open(t, O_RDONLY, 0);
      if (fd >= 0) {
        void* m = mmap(nullptr, 1u << 20, PROT_READ, MAP_SHARED, fd, 0);
        close(fd);
        if (m != MAP_FAILED) g.shard_table = static_cast<const uint8_t*>(m);
      }
    }
  }
  void* const r0 = g.ring.load(std::memory_order_acquire);
  g.rec32 = r0 && mislo_ring_rec_size(r0) == 32;
  g.rec24 = r0 && mislo_ring_rec_size(r0) == 24;
  g.rec16 = r0 && mislo_ring_rec_size(r0) == 16;
  g.pod = (uint32_t)env_u64("MISLO_POD_ID", 0);
  route();
  g.node = (uint16_t)env_u64("MISLO_NODE_ID", 0);
  g.svc = (uint16_t)env_u64("MISLO_SVC_ID", 0);
  g.hbm_bytes = env_u64("MISLO_HBM_BYTES", 288ull << 30);
  g.max_eps = env_u64("MISLO_MAX_EPS", 200000);
  g.queue_floor_ns = env_u64("MISLO_QUEUE_FLOOR_NS", 10000000);
  g.xgmi_bytes_per_ns = (double)env_u64("MISLO_XGMI_GBPS", 64);  // GB/s == bytes/ns
  g.verbose = env_u64("MISLO_ROCPROF_VERBOSE", 0) != 0;
  if (const char* ps = std::getenv("MISLO_PCI_SYSFS")) g.pci_sysfs = ps;
  g.hbm_sample_ms = env_u64("MISLO_HBM_SAMPLE_MS", 1000);
  g.foreign_ms = env_u64("MISLO_FOREIGN_MS", 100);
  g.foreign_floor_pct = env_u64("MISLO_FOREIGN_FLOOR_PCT", 10);
  g.foreign_min_hot = env_u64("MISLO_FOREIGN_MIN_HOT", 2);
  g.occ_ms = std::max<uint64_t>(1, env_u64("MISLO_OCC_MS", 10));
  g.foreign_min_samples = env_u64("MISLO_FOREIGN_MIN_SAMPLES", 3);
  g.wait_needs_foreign = env_u64("MISLO_WAIT_NEEDS_FOREIGN", 1) != 0;
  if (const char* kp = std::getenv("MISLO_KFD_PROC")) g.kfd_proc = kp;
  g.kfd_dir = access(g.kfd_proc.c_str(), R_OK | X_OK) == 0;
  rocprofiler_query_available_agents(ROCPROFILER_AGENT_INFO_VERSION_0, agents_cb, sizeof(rocprofiler_agent_v0_t),
                                     nullptr);
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
  if (g.hbm_sample_ms || g.foreign_ms) g.sampler = std::thread(sampler_main);
  if (g.verbose)
    std::fprintf(stderr, "[mislo-rocprof] started (ring=%s attached=%d)\n", name ? name : "/mislo-agent-events",
                 g.ring.load() != nullptr);
  return ok ? 0 : -1;
}

void tool_fini(void*) {
  {
    std::lock_guard<std::mutex> lk(g.smu);
    g.stop = true;
  }
  g.scv.notify_all();
  if (g.sampler.joinable()) g.sampler.join();
  rocprofiler_flush_buffer(g.buffer);
  if (g.verbose)
    std::fprintf(stderr, "[mislo-rocprof] pushed=%llu dropped=%llu\n", (unsigned long long)g.pushed.load(),
                 (unsigned long long)g.dropped.load());
  g.ring.store(nullptr, std::memory_order_release);  // no emit() picks a ring about to close
  for (void* r : g.rings)
    if (r) mislo_ring_close(r);
  g.rings.clear();
}

}  // namespace

extern "C" {

// Counters for tests / the agent's ring statistics.
uint64_t mislo_rocprof_pushed() { return g.pushed.load(); }
uint64_t mislo_rocprof_dropped() { return g.dropped.load(); }

// The calling thread's current request trace (0 = none): kernels it enqueues from now on carry it.
void mislo_rocprof_set_trace(uint64_t trace_h) { t_trace = trace_h; }

// The last decided foreign-time interval of the GPU agent with the given index: the share of idle
// readings with other processes' waves on the GPU and their mean occupancy (CUs); returns the
// intervals decided so far (-1: no such GPU).
int64_t mislo_rocprof_foreign(int gpu_index, double* share, double* occ_mean) {
  int i = 0;
  for (auto& kv : g.occ) {
    if (i++ != gpu_index) continue;
    *share = kv.second.share;
    *occ_mean = kv.second.occ_mean;
    return (int64_t)kv.second.decisions;
  }
  return -1;
}

// Dispatch waits (>= the queue floor) on the GPU agent with the given index: emitted (foreign waves
// seen during the wait, or occupancy unreadable) and withheld; -1 for an unknown index.
int64_t mislo_rocprof_waits(int gpu_index, uint64_t* emitted, uint64_t* unconfirmed) {
  int i = 0;
  std::lock_guard<std::mutex> lk(g.mu);
  for (auto& kv : g.occ) {
    if (i++ != gpu_index) continue;
    *emitted = kv.second.waits_emitted;
    *unconfirmed = kv.second.waits_unconfirmed;
    return 0;
  }
  return -1;
}

// This process's own KFD entry (host pid; 0 = not identified yet) on the GPU agent with the given
// index, and the idle / in-flight readings it was learned from.
int64_t mislo_rocprof_self(int gpu_index, uint64_t* idle_n, uint64_t* busy_n) {
  int i = 0;
  for (auto& kv : g.occ) {
    if (i++ != gpu_index) continue;
    *idle_n = kv.second.idle_n;
    *busy_n = kv.second.busy_n;
    return kv.second.self_pid;
  }
  return -1;
}

// The occupancy readings' cost on the GPU agent with the given index: readings, their total time
// (ns) and the readings not counted because a kernel of this process was in flight (before its
// own entry was identified).
int64_t mislo_rocprof_occ_cost(int gpu_index, uint64_t* reads, uint64_t* read_ns, uint64_t* busy_skips) {
  int i = 0;
  for (auto& kv : g.occ) {
    if (i++ != gpu_index) continue;
    *reads = kv.second.reads;
    *read_ns = kv.second.read_ns;
    *busy_skips = kv.second.busy_skips;
    return 0;
  }
  return -1;
}

// Node-wide HBM pressure (milli-pct) of the GPU agent with the given index among the GPUs
// (-1 if its sysfs counters are unreadable), for tests and the agent's checks.
int64_t mislo_rocprof_hbm_milli(int gpu_index) {
  int i = 0;
  for (auto& kv : g.vram) {
    if (i++ != gpu_index) continue;
    if (kv.second.used_fd < 0 || kv.second.total_fd < 0) return -1;
    const uint64_t total = read_u64_fd(kv.second.total_fd);
    return total ? (int64_t)((double)read_u64_fd(kv.second.used_fd) * 100000.0 / (double)total) : -1;
  }
  return -1;
}

// A GPU pair's calibration (xGMI): copies seen, calibrated bytes/ns (0 = no large copy yet) and
// the smallest small-copy latency (ns; ~0 = none). Returns the number of calibrated pairs.
int mislo_rocprof_links(int i, uint64_t* copies, double* bytes_per_ns, uint64_t* min_small_ns) {
  std::lock_guard<std::mutex> lk(g.mu);
  int j = 0;
  for (auto& kv : g.links) {
    if (j++ == i) {
      *copies = kv.second.copies;
      *bytes_per_ns = kv.second.bytes_per_ns;
      *min_small_ns = kv.second.min_small_ns;
    }
  }
  return (int)g.links.size();
}

rocprofiler_tool_configure_result_t* rocprofiler_configure(uint32_t, const char*, uint32_t,
                                                           rocprofiler_client_id_t* id) {
  id->name = "llm-slo-ebpf-toolkit-amd";
  g.client = id;
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init,
                                                 &tool_fini, nullptr};
  return &cfg;
}

}  // extern "C"
