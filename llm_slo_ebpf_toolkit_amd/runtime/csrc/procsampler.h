// Native unprivileged CPU / memory signal sampler: the agent's kernel-signal producer where BPF is
// not allowed (collector/procfs.py is the Python model of exactly this code and the oracle of its
// tests). A thread of the agent reads, every interval, for each watched process:
//
//   /proc/<pid>/task/<tid>/schedstat   on-CPU ns, run-queue wait ns, timeslices of each thread
//   <cgroup>/cpu.stat                  throttled_usec (v2) / throttled_time (v1) of the nearest
//                                      ancestor group with a CPU quota (CFS bandwidth throttling)
//   <cgroup>/memory.pressure           PSI "some" total (v2; else the node's /proc/pressure/memory)
//   <cgroup>/cpu.pressure              PSI "some" total (opt-in: only meaningful for a pod-private group)
//
// and pushes records straight into the agent's user-space ring in its record size (USER24 /
// USER32 / EVENT), stamped with the process's pid in its own pid namespace and its pod id:
//
//   type 3  runqueue_delay_ms  mean run-queue wait per timeslice over the threads whose mean
//                              reached the floor (runqueue_delay.bpf.c: per-wakeup waits >= 100 us)
//   type 6  cpu_steal_pct      CPU time the process was runnable but not running over the
//                              interval, in percent of one CPU (sum over its threads of the
//                              run-queue wait / interval): the process's view of stolen CPU. Under
//                              EEVDF a starved thread waits a short time per wakeup but most of the
//                              interval in total, so this fires where the per-wakeup mean does not.
//                              Emitted once the share has stayed at the floor for steal_sustain
//                              intervals in a row: a service's own threads spike past it now and then.
//                              Where the pod runs on a small CPU set (Cpus_allowed_list of at most
//                              steal_foreign_max_cpus), the wait counts only while other processes
//                              kept those CPUs busy (/proc/stat busy time minus the pod's own on-CPU
//                              time, at least steal_foreign_milli of their capacity): a pod catching
//                              up on its own backlog waits behind its own threads, not a neighbour
//   type 7  mem_reclaim_latency_ms  PSI memory stall of the process's group over the interval
//   type 12 cfs_throttled_ms   CFS bandwidth throttling of the process's quota group over the interval
//
// Each signal has an emit floor (the BPF probes' in-kernel filters); the overhead guard sheds by
// clearing a signal's bit in the mask or pausing the sampler (agent/daemon.py _guard_tick).
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

struct ProcSamplerConfig {
  std::string proc_root = "/proc";
  std::string cgroup_root = "/sys/fs/cgroup";
  uint32_t node_id = 0;
  uint64_t runq_floor_ns = 100000;    // runqueue_delay.bpf.c emit floor (100 us per timeslice)
  uint64_t steal_floor_milli = 20000; // 20 % of one CPU over the interval (collector/procfs.py STEAL_FLOOR_MILLI)
  uint32_t steal_sustain = 3;         // ... in this many consecutive intervals (procfs.py STEAL_SUSTAIN)
  uint64_t cfs_floor_ns = 100000;
  uint64_t mem_floor_ns = 100000;
  bool cgroup_cpu_psi = false;        // cpu_steal_pct = max(wait share, the group's cpu.pressure share)
  uint64_t steal_foreign_milli = 25000;  // neighbours' share of the pod's CPUs a wait needs (0: no gate)
  uint32_t steal_foreign_max_cpus = 32;  // pods on larger CPU sets are not gated (node-wide load says little)
};

constexpr uint16_t kSigRunq = 3, kSigSteal = 6, kSigMem = 7, kSigCfs = 12;
constexpr uint32_t kProcAllSignals = (1u << kSigRunq) | (1u << kSigSteal) | (1u << kSigMem) | (1u << kSigCfs);

struct ProcSamplerStats {
  uint64_t ticks = 0, emitted = 0, dropped = 0, targets = 0, last_tick_ns = 0, max_tick_ns = 0;
  uint64_t by_type[4] = {0, 0, 0, 0};  // runq, steal, mem, cfs
  uint64_t cfs_groups = 0;             // quota groups found for the targets (0: throttling unobservable)
  uint64_t steal_gated = 0;            // intervals a wait share at the floor was not counted (no neighbour load)
};

class ProcSampler {
 public:
  // `ring` may be null (tick() then only returns the records); it must outlive the sampler.
  ProcSampler(Ring* ring, ProcSamplerConfig cfg);
  ~ProcSampler();
  ProcSampler(const ProcSampler&) = delete;
  ProcSampler& operator=(const ProcSampler&) = delete;

  void set_targets(const std::vector<std::pair<uint32_t, uint32_t>>& pid_pod);
  // One interval at (realtime ns, monotonic ns): the records it produced (pushed when a ring is set).
  std::vector<EventRec> tick(int64_t wall_ns, uint64_t mono_ns);
  void start(uint64_t interval_ns);
  void stop();
  void set_mask(uint32_t mask) { mask_.store(mask, std::memory_order_relaxed); }
  uint32_t mask() const { return mask_.load(std::memory_order_relaxed); }
  void set_paused(bool p) { paused_.store(p, std::memory_order_relaxed); }
  bool paused() const { return paused_.load(std::memory_order_relaxed); }
  ProcSamplerStats stats();
  ProcSamplerConfig& config() { return cfg_; }

 private:
  struct Group {  // a cgroup file's last reading
    uint64_t last = 0, delta = 0;
    bool have = false, seen = false;
  };
  struct Proc {
    uint32_t ns_pid = 0;
    uint32_t steal_run = 0;  // consecutive intervals with the wait share at the floor
    bool resolved = false;
    // its threads' schedstat files, kept open (one pread per thread and tick instead of an
    // open / read / close); the task directory is re-listed every task_rescan_ns
    std::vector<std::pair<uint32_t, int>> task_fds;  // (tid, fd), tid order
    uint64_t listed_ns = 0;
    bool listed = false;
    std::string cfs_file, mem_file, cpu_psi_file;  // empty: none
    std::vector<uint32_t> cpus;  // Cpus_allowed_list (empty: unknown)
  };
  struct Tid {  // a thread's last schedstat reading
    uint64_t run = 0, wait = 0, slices = 0;
  };
  void resolve(uint32_t pid, Proc& p);
  void list_tasks(uint32_t pid, Proc& p, uint64_t mono_ns);
  static void close_tasks(Proc& p);
  uint64_t task_rescan_ns_ = 1000000000;
  uint64_t group_delta(const std::string& file, int kind);  // kind 0: cpu.stat throttle ns, 1: PSI some ns

  Ring* ring_;
  ProcSamplerConfig cfg_;
  std::mutex mu_;  // targets_, state, stats
  std::vector<std::pair<uint32_t, uint32_t>> targets_;
  std::map<std::pair<uint32_t, uint32_t>, Tid> prev_;  // (pid, tid) -> last reading
  std::vector<uint64_t> cpu_busy_;                   // /proc/stat busy jiffies per CPU, last tick
  bool cpu_busy_have_ = false;
  uint64_t cpu_busy_tick_ = 0;                       // the tick that read cpu_busy_
  bool read_cpu_busy(std::vector<uint64_t>* out);
  std::map<uint32_t, Proc> procs_;
  std::map<std::string, Group> groups_;
  uint64_t prev_mono_ = 0;
  ProcSamplerStats st_;
  std::atomic<uint32_t> mask_{kProcAllSignals};
  std::atomic<bool> paused_{false};
  std::thread thr_;
  std::mutex tmu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

}  // namespace mislo
