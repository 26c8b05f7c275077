// Native KFD sampler (gpusampler.h).
#include "gpusampler.h"

#include <dirent.h>
#include <fcntl.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <set>

#include "bpfsys.h"
#include "fsread.h"

namespace mislo {

GpuSampler::GpuSampler(Ring* ring, GpuSamplerConfig cfg) : ring_(ring), cfg_(std::move(cfg)) {}

GpuSampler::~GpuSampler() {
  stop();
  for (auto& kv : occ_fd_) ::close(kv.second);
}

void GpuSampler::set_targets(const std::vector<std::pair<uint32_t, uint32_t>>& pid_pod) {
  std::lock_guard<std::mutex> lk(mu_);
  targets_ = pid_pod;
  refresh_locked();
}

void GpuSampler::set_hip_activity(uint32_t pid, const HipActivity& a) {
  std::lock_guard<std::mutex> lk(mu_);
  hip_override_[pid] = a;
}

// Which GPUs each watched process has a KFD stats directory for (it opened them).
void GpuSampler::refresh_locked() {
  std::map<uint32_t, Proc> live;
  std::vector<uint64_t> gpus;
  for (const auto& tp : targets_) {
    const uint32_t pid = tp.first;
    auto it = procs_.find(pid);
    Proc p = it != procs_.end() ? it->second : Proc{};
    if (!p.resolved) {
      p.ns_pid = ns_pid_of(cfg_.proc_root, pid);
      p.resolved = true;
    }
    p.gpus.clear();
    const std::string dir = join(cfg_.kfd_proc, std::to_string(pid));
    if (DIR* d = ::opendir(dir.c_str())) {
      while (dirent* e = ::readdir(d)) {
        if (std::strncmp(e->d_name, "stats_", 6) != 0) continue;
        const uint64_t g = std::strtoull(e->d_name + 6, nullptr, 10);
        if (g) p.gpus.push_back(g);
      }
      ::closedir(d);
    }
    std::sort(p.gpus.begin(), p.gpus.end());
    gpus.insert(gpus.end(), p.gpus.begin(), p.gpus.end());
    live[pid] = std::move(p);
  }
  std::sort(gpus.begin(), gpus.end());
  gpus.erase(std::unique(gpus.begin(), gpus.end()), gpus.end());
  procs_.swap(live);
  if (gpus != gpus_) last_scan_ns_ = 0;  // other GPUs watched: re-open the files at the next reading
  gpus_.swap(gpus);
}

void GpuSampler::rescan_locked() {
  std::map<std::pair<uint32_t, uint64_t>, int> next;
  if (DIR* d = ::opendir(cfg_.kfd_proc.c_str())) {
    char path[512];
    while (dirent* e = ::readdir(d)) {
      if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
      const uint32_t pid = (uint32_t)std::strtoul(e->d_name, nullptr, 10);
      for (uint64_t g : gpus_) {
        const auto key = std::make_pair(pid, g);
        const auto it = occ_fd_.find(key);
        if (it != occ_fd_.end()) {  // still listed: keep its open file
          next[key] = it->second;
          occ_fd_.erase(it);
          continue;
        }
        std::snprintf(path, sizeof(path), "%s/%s/stats_%llu/cu_occupancy", cfg_.kfd_proc.c_str(), e->d_name,
                      (unsigned long long)g);
        const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
        if (fd >= 0) next[key] = fd;
      }
    }
    ::closedir(d);
  }
  for (auto& kv : occ_fd_) ::close(kv.second);  // processes gone, GPUs no longer watched
  occ_fd_.swap(next);
  ++st_.scans;
}

void GpuSampler::sample() {
  const auto t0 = std::chrono::steady_clock::now();
  std::lock_guard<std::mutex> lk(mu_);
  if (gpus_.empty() || !enabled()) return;
  const uint64_t now = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                           t0.time_since_epoch()).count();
  if (!last_scan_ns_ || now - last_scan_ns_ >= rescan_ns_) {
    rescan_locked();
    last_scan_ns_ = now;
  }
  std::map<uint32_t, uint32_t> pod_of;
  for (const auto& tp : targets_) pod_of[tp.first] = tp.second;
  // every KFD process's occupancy of the watched GPUs
  std::vector<uint64_t> total(gpus_.size(), 0);
  std::map<std::pair<uint32_t, uint64_t>, uint64_t> own;  // (pod, gpu) -> its processes' occupancy
  for (auto it = occ_fd_.begin(); it != occ_fd_.end();) {
    uint64_t occ = 0;
    if (!pread_u64(it->second, &occ)) {  // the process is gone
      ::close(it->second);
      it = occ_fd_.erase(it);
      continue;
    }
    ++st_.reads;
    const size_t i = (size_t)(std::lower_bound(gpus_.begin(), gpus_.end(), it->first.second) - gpus_.begin());
    if (i < gpus_.size() && gpus_[i] == it->first.second) {
      total[i] += occ;
      const auto pp = pod_of.find(it->first.first);
      if (pp != pod_of.end()) own[{pp->second, gpus_[i]}] += occ;
    }
    ++it;
  }
  // each (pod, GPU) the pod's processes have opened: one reading
  std::set<std::pair<uint32_t, uint64_t>> pairs;
  for (const auto& tp : targets_) {
    const auto pr = procs_.find(tp.first);
    if (pr != procs_.end())
      for (uint64_t g : pr->second.gpus) pairs.insert({tp.second, g});
  }
  for (const auto& key : pairs) {
    const size_t gi = (size_t)(std::lower_bound(gpus_.begin(), gpus_.end(), key.second) - gpus_.begin());
    const auto oi = own.find(key);
    const uint64_t mine = oi != own.end() ? oi->second : 0;
    const uint64_t foreign = total[gi] > mine ? total[gi] - mine : 0;
    Acc& a = acc_[key];
    ++a.samples;
    a.hot += foreign > 0;
    a.own_hot += mine > 0;
    a.foreign_sum += (double)foreign;
  }
  ++st_.samples;
  const uint64_t took = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now() - t0).count();
  st_.read_ns += took;
  if (took > st_.max_sample_ns) st_.max_sample_ns = took;
}

// gpu_queue_delay_ms not shed: by this sampler's mask, or the ring's drop mask (the overhead
// guard's GPU step, the one every GPU producer of the ring obeys)
bool GpuSampler::enabled() const {
  if (!(mask_.load(std::memory_order_relaxed) >> kSigGpuQueue & 1)) return false;
  return !ring_ || !(ring_->header()->drop_mask.load(std::memory_order_relaxed) >> kSigGpuQueue & 1);
}

bool GpuSampler::hip_locked(uint32_t pid, HipActivity* a) {
  const int fd = hip_fd_.load(std::memory_order_relaxed);
  if (fd >= 0) return bpf_map_lookup(fd, &pid, a) == 0;
  const auto it = hip_override_.find(pid);
  if (it == hip_override_.end()) return false;
  *a = it->second;
  return true;
}

std::vector<EventRec> GpuSampler::decide(int64_t wall_ns, uint64_t mono_ns) {
  std::vector<EventRec> out;
  std::lock_guard<std::mutex> lk(mu_);
  const uint32_t mask = enabled() ? 1u << kSigGpuQueue : 0u;
  const uint64_t dt = prev_mono_ && mono_ns > prev_mono_ ? mono_ns - prev_mono_ : 0;
  prev_mono_ = mono_ns;
  const uint32_t n_st = std::max<uint32_t>(1u, cfg_.stamps);
  auto rec = [&](uint32_t ns_pid, uint32_t pid, uint32_t pod, uint64_t value) {
    for (uint32_t i = 0; i < n_st; ++i) {  // sub-interval i's middle; the value split evenly
      EventRec e{};
      e.ts_ns = wall_ns - (int64_t)dt + (int64_t)((2 * (uint64_t)i + 1) * dt / (2 * (uint64_t)n_st));
      e.value = value / n_st;
      e.pid = ns_pid;
      e.tid = pid;
      e.pod_id = pod;
      e.node_id = (uint16_t)cfg_.node_id;
      e.signal_type = kSigGpuQueue;
      e.flags = 1u << 8;  // has_gpu
      out.push_back(e);
    }
  };
  // the pods whose HIP runtime submitted work or waited on the GPU since the last decision, and
  // how long their threads waited: ROCr's completion-signal waits (every blocking HIP path ends in
  // one) when those uprobes report, else the HIP synchronize and copy calls
  std::map<uint32_t, bool> hip_active;
  std::map<uint32_t, uint64_t> pod_wait;
  // pods whose uprobes report: a measured wait of 0 is "did not block", not "no measurement"
  std::map<uint32_t, bool> pod_reports;
  std::map<uint32_t, HipActivity> hip_now;
  for (const auto& tp : targets_) {
    HipActivity a;
    if (!hip_locked(tp.first, &a)) continue;
    hip_now[tp.first] = a;
    if (a.waits || a.syncs) pod_reports[tp.second] = true;  // the wait / synchronize uprobes have fired
    const auto pv = hip_prev_.find(tp.first);
    if (pv == hip_prev_.end()) continue;
    const HipActivity& b = pv->second;
    const uint64_t wait = a.waits != b.waits || a.wait_ns != b.wait_ns
                              ? a.wait_ns - b.wait_ns
                              : (a.sync_ns - b.sync_ns) + (a.copy_ns - b.copy_ns);
    if (a.launches != b.launches || a.copies != b.copies || wait) hip_active[tp.second] = true;
    if (wait) pod_wait[tp.second] += wait;
  }
  hip_prev_.swap(hip_now);
  last_.clear();
  for (const auto& kv : acc_) {
    const Acc& a = kv.second;
    if (a.samples < cfg_.min_samples) continue;
    GpuShare s;
    s.pod = kv.first.first;
    s.gpu_id = kv.first.second;
    s.samples = a.samples, s.hot = a.hot, s.own_hot = a.own_hot;
    s.share = (double)a.hot / (double)a.samples;
    s.foreign_mean = a.foreign_sum / (double)a.samples;
    s.active = a.own_hot > 0 || hip_active.count(s.pod);
    uint32_t& hold = hold_[kv.first];
    if (s.active) {
      hold = cfg_.starved_hold;
    } else if (hold && s.share * 100.0 >= (double)cfg_.starved_pct) {
      s.active = s.starved = true;
      --hold;
    } else {
      hold = 0;
    }
    const auto pw = pod_wait.find(s.pod);
    s.gpu_wait_ns = pw != pod_wait.end() ? pw->second : 0;
    s.wait_reported = pod_reports.count(s.pod) > 0;
    ++st_.decisions;
    if (dt && s.active && (mask >> kSigGpuQueue & 1) && s.share * 100.0 >= (double)cfg_.floor_pct) {
      // the pod's measured GPU wait, the share of it other processes held the GPU (a pod that did
      // not block this interval: 0); without the uprobes, the share of the interval (ADVICE r5:
      // a 0 wait no longer jumps to the whole interval)
      const uint64_t base = s.wait_reported ? std::min<uint64_t>(s.gpu_wait_ns, dt) : dt;
      const uint64_t v = (uint64_t)(s.share * (double)base);
      // stamped with the pod's first process on that GPU
      for (const auto& tp : targets_) {
        if (tp.second != s.pod) continue;
        const auto pr = procs_.find(tp.first);
        if (pr == procs_.end() || !std::binary_search(pr->second.gpus.begin(), pr->second.gpus.end(), s.gpu_id))
          continue;
        rec(pr->second.ns_pid, tp.first, s.pod, v);
        s.delay_ns = v;
        break;
      }
    }
    last_.push_back(s);
  }
  // queue evictions: growth of each process's evicted_ms per GPU
  char path[512];
  for (const auto& tp : targets_) {
    auto pr = procs_.find(tp.first);
    if (pr == procs_.end()) continue;
    Proc& p = pr->second;
    for (uint64_t g : p.gpus) {
      std::snprintf(path, sizeof(path), "%s/%u/stats_%llu/evicted_ms", cfg_.kfd_proc.c_str(), tp.first,
                    (unsigned long long)g);
      uint64_t ms = 0;
      if (!read_u64_file(path, &ms)) continue;
      auto ev = p.evicted_ms.find(g);
      const bool primed = ev != p.evicted_ms.end();
      const uint64_t d = primed && ms > ev->second ? ms - ev->second : 0;
      p.evicted_ms[g] = ms;
      if (!d) continue;
      ++st_.evictions;
      if (cfg_.evictions && dt && (mask >> kSigGpuQueue & 1) && d * 1000000ull >= cfg_.evict_floor_ns)
        rec(p.ns_pid, tp.first, tp.second, d * 1000000ull);
    }
  }
  st_.pairs = acc_.size();
  for (auto it = hold_.begin(); it != hold_.end();)  // only pairs read this interval keep a hold
    it = it->second && acc_.count(it->first) ? std::next(it) : hold_.erase(it);
  acc_.clear();
  refresh_locked();
  uint64_t pushed = 0;
  if (ring_ && !out.empty()) {
    const uint32_t rs = ring_->rec_size();
    std::vector<uint8_t> buf(2 * out.size() * rs);  // a traced USER16 record takes two slots
    size_t n = 0, recs = 0;
    for (const EventRec& e : out) {
      const int w = pack_user(e, rs, buf.data() + n * rs);
      n += (size_t)w;
      recs += w ? 1u : 0u;
    }
    pushed = n && ring_->push_batch(buf.data(), n) == n ? recs : 0;  // all or nothing
    st_.emitted += pushed;
    st_.dropped += out.size() - pushed;
  } else {
    st_.emitted += out.size();
  }
  return out;
}

void GpuSampler::start(uint64_t sample_ns, uint64_t decide_ns) {
  stop();
  {
    std::lock_guard<std::mutex> lk(tmu_);
    stop_ = false;
  }
  thr_ = std::thread([this, sample_ns, decide_ns] {
    std::unique_lock<std::mutex> lk(tmu_);
    uint64_t next_decide = 0;
    while (!cv_.wait_for(lk, std::chrono::nanoseconds(sample_ns), [this] { return stop_; })) {
      if (paused_.load(std::memory_order_relaxed)) continue;
      lk.unlock();
      sample();
      timespec rt{}, mo{};
      clock_gettime(CLOCK_MONOTONIC, &mo);
      const uint64_t mono = (uint64_t)mo.tv_sec * 1000000000ull + (uint64_t)mo.tv_nsec;
      if (mono >= next_decide) {
        next_decide = mono + decide_ns;
        clock_gettime(CLOCK_REALTIME, &rt);
        decide((int64_t)rt.tv_sec * 1000000000ll + rt.tv_nsec, mono);
      }
      lk.lock();
    }
  });
}

void GpuSampler::stop() {
  {
    std::lock_guard<std::mutex> lk(tmu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (thr_.joinable()) thr_.join();
}

GpuSamplerStats GpuSampler::stats() {
  std::lock_guard<std::mutex> lk(mu_);
  return st_;
}

std::vector<GpuShare> GpuSampler::shares() {
  std::lock_guard<std::mutex> lk(mu_);
  return last_;
}

}  // namespace mislo
