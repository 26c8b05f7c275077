// Native KFD sampler: the agent's view of who holds each GPU, for pods whose workloads were not
// started with the rocprofiler tool (probes/rocprof). The amdgpu KFD driver publishes, per process
// (directory named by its host pid) and per GPU (KFD gpu_id):
//
//   /sys/class/kfd/kfd/proc/<pid>/stats_<gpu_id>/cu_occupancy   CU-equivalents of the process's
//                                                                 waves resident on the GPU now
//   /sys/class/kfd/kfd/proc/<pid>/stats_<gpu_id>/evicted_ms      total time its queues were evicted
//
// readable without privileges. A thread samples every process's occupancy of the GPUs the
// watched pods use (default every 20 ms) and, each decision interval (default 500 ms), for every
// (pod, GPU):
//
//   type 13 gpu_queue_delay_ms  the share of readings at which OTHER processes (not the pod's
//                               own) held waves on that GPU, as ns of the interval, when the pod
//                               was using the GPU (its own waves were seen, or its HIP runtime
//                               submitted work or waited on the GPU: gpu_kfd.bpf.c hip_activity)
//                               and the share reached the floor (default 10 %). Where the HIP /
//                               ROCr uprobes report how long the pod's threads waited on the GPU
//                               (ROCr completion-signal waits; else hip*Synchronize + hipMemcpy
//                               call time), the value is that share of the wait (capped at the
//                               interval): the delay the pod actually sat through
//   type 13 gpu_queue_delay_ms  the time the pod's queues were evicted over the interval
//                               (evicted_ms growth; the BPF probe's kfd_process_evict_queues ->
//                               restore span, for nodes without BPF) when >= 1 ms
//
// The host pids in the KFD tree are the agent's own pids only when it runs in the host pid
// namespace (the DaemonSet's hostPID: true); records are stamped with the process's pid in its own
// namespace and its pod id, like the procfs sampler's (procsampler.h). A workload inside a
// container without the agent's pid namespace is covered by the in-process tool instead, which
// reads the same files while it has no kernel in flight (mislo_rocprof.cpp foreign time).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "records.h"
#include "ring.h"

namespace mislo {

struct GpuSamplerConfig {
  std::string kfd_proc = "/sys/class/kfd/kfd/proc";
  std::string proc_root = "/proc";
  uint32_t node_id = 0;
  uint64_t floor_pct = 10;             // foreign share of the interval to emit
  uint64_t min_samples = 3;            // readings of a (pod, GPU) needed to decide an interval
  uint64_t evict_floor_ns = 1000000;   // eviction time per interval to emit
  bool evictions = true;               // evicted_ms records (off when gpu_kfd.bpf.c's kprobes run)
  // a pod active last interval that shows no occupancy of its own while other processes hold the
  // GPU in >= starved_pct % of the readings is starved, not idle (its kernels wait for CUs and
  // cu_occupancy only counts resident waves): it stays active for up to starved_hold intervals
  uint32_t starved_hold = 2;
  uint64_t starved_pct = 90;
  // records per contended interval: the interval's delay split evenly over this many records
  // stamped at the sub-intervals' middles, so a request span's pod+pid join (100 ms of its start)
  // finds one wherever its start falls; the floor still gates on the whole interval's share
  uint32_t stamps = 1;
};

// gpu_kfd.bpf.c hip_activity value (probes/ebpf/mislo_record.h struct mislo_hip_act)
struct HipActivity {
  uint64_t launches = 0, copies = 0, last_ns = 0, sync_ns = 0, syncs = 0;
  uint64_t copy_ns = 0, wait_ns = 0, waits = 0;  // hipMemcpy(Async) call time, ROCr signal waits
};
static_assert(sizeof(HipActivity) == 64, "mislo_hip_act layout");

constexpr uint16_t kSigGpuQueue = 13;

struct GpuSamplerStats {
  uint64_t samples = 0, reads = 0, read_ns = 0, decisions = 0, emitted = 0, dropped = 0, evictions = 0, scans = 0;
  uint64_t max_sample_ns = 0;
  uint64_t pairs = 0;  // (pod, GPU) pairs seen at the last decision
};

// One (pod, GPU) pair's last decided interval (tests, metrics).
struct GpuShare {
  uint32_t pod = 0;
  uint64_t gpu_id = 0;
  uint64_t samples = 0, hot = 0, own_hot = 0;
  double share = 0.0, foreign_mean = 0.0;
  bool active = false;
  bool starved = false;      // active by the starvation hold, not by its own readings
  uint64_t gpu_wait_ns = 0;  // the pod's host-side GPU wait over the interval
  bool wait_reported = false;  // the pod's HIP / ROCr uprobes report (gpu_wait_ns is measured, 0 included)
  uint64_t delay_ns = 0;     // the gpu_queue_delay_ms value decided (0: none emitted)
};

class GpuSampler {
 public:
  GpuSampler(Ring* ring, GpuSamplerConfig cfg);
  ~GpuSampler();
  GpuSampler(const GpuSampler&) = delete;
  GpuSampler& operator=(const GpuSampler&) = delete;

  // (host pid, pod id) of the watched processes
  void set_targets(const std::vector<std::pair<uint32_t, uint32_t>>& pid_pod);
  // the pinned gpu_kfd hip_activity map (-1: none; the sampler does not own the fd)
  void set_hip_map(int fd) { hip_fd_.store(fd, std::memory_order_relaxed); }
  // tests / non-BPF producers: a process's HIP activity counters, used when no map is set
  void set_hip_activity(uint32_t pid, const HipActivity& a);
  // One occupancy reading of the watched pods' GPUs.
  void sample();
  // End of a decision interval at (realtime ns, monotonic ns): the records it produced (pushed
  // when a ring is set).
  std::vector<EventRec> decide(int64_t wall_ns, uint64_t mono_ns);
  void start(uint64_t sample_ns, uint64_t decide_ns);
  void stop();
  void set_mask(uint32_t mask) { mask_.store(mask, std::memory_order_relaxed); }
  uint32_t mask() const { return mask_.load(std::memory_order_relaxed); }
  void set_paused(bool p) { paused_.store(p, std::memory_order_relaxed); }
  bool paused() const { return paused_.load(std::memory_order_relaxed); }
  GpuSamplerStats stats();
  std::vector<GpuShare> shares();

 private:
  struct Acc {  // one (pod, GPU) pair's readings in the current interval
    uint64_t samples = 0, hot = 0, own_hot = 0;
    double foreign_sum = 0.0;
  };
  struct Proc {
    uint32_t ns_pid = 0;
    std::vector<uint64_t> gpus;  // KFD gpu_ids it has a stats directory for
    std::map<uint64_t, uint64_t> evicted_ms;  // gpu_id -> last evicted_ms reading
    bool resolved = false;
  };
  void refresh_locked();  // target processes' GPUs (each decision)
  void rescan_locked();   // the KFD process tree: open the watched GPUs' cu_occupancy files
  bool hip_locked(uint32_t pid, HipActivity* a);
  bool enabled() const;

  Ring* ring_;
  GpuSamplerConfig cfg_;
  std::mutex mu_;
  std::vector<std::pair<uint32_t, uint32_t>> targets_;
  std::map<uint32_t, Proc> procs_;                         // target pid -> state
  std::vector<uint64_t> gpus_;                             // gpu_ids any target uses
  // (KFD pid, gpu_id) -> its cu_occupancy file, kept open between readings (one pread each:
  // opening every process's file per reading cost ~100 us at 50 readings/s); the tree is
  // re-listed every rescan_ns for processes that came and went
  std::map<std::pair<uint32_t, uint64_t>, int> occ_fd_;
  uint64_t last_scan_ns_ = 0;
  uint64_t rescan_ns_ = 500000000;
  std::map<std::pair<uint32_t, uint64_t>, Acc> acc_;       // (pod, gpu) -> readings
  std::map<std::pair<uint32_t, uint64_t>, uint32_t> hold_;  // (pod, gpu) -> starvation hold left
  std::map<uint32_t, HipActivity> hip_prev_, hip_override_;
  std::vector<GpuShare> last_;
  uint64_t prev_mono_ = 0;
  GpuSamplerStats st_;
  std::atomic<int> hip_fd_{-1};
  std::atomic<uint32_t> mask_{1u << kSigGpuQueue};
  std::atomic<bool> paused_{false};
  std::thread thr_;
  std::mutex tmu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

}  // namespace mislo
