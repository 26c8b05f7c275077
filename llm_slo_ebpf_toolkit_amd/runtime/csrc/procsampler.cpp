// Native unprivileged CPU / memory sampler (procsampler.h). collector/procfs.py SchedstatSampler is
// the Python model of this file, record for record.
#include "procsampler.h"

#include "fsread.h"

#include <dirent.h>
#include <fcntl.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>

namespace mislo {

namespace {

bool readable(const std::string& path) { return ::access(path.c_str(), R_OK) == 0; }

std::string parent(const std::string& d) {
  const size_t k = d.find_last_of('/');
  return k == std::string::npos || k == 0 ? std::string("/") : d.substr(0, k);
}

// "name value" line of a flat-keyed file (cpu.stat)
bool keyed_u64(const std::string& text, const char* key, uint64_t* v) {
  const size_t kl = std::strlen(key);
  size_t pos = 0;
  while (pos < text.size()) {
    size_t e = text.find('\n', pos);
    if (e == std::string::npos) e = text.size();
    if (e - pos > kl && text.compare(pos, kl, key) == 0 && text[pos + kl] == ' ') {
      *v = std::strtoull(text.c_str() + pos + kl + 1, nullptr, 10);
      return true;
    }
    pos = e + 1;
  }
  return false;
}

// PSI "some ... total=<us>"
bool psi_some_us(const std::string& text, uint64_t* v) {
  if (text.compare(0, 4, "some") != 0) return false;
  const size_t e = text.find('\n');
  const size_t t = text.rfind("total=", e == std::string::npos ? text.size() : e);
  if (t == std::string::npos) return false;
  *v = std::strtoull(text.c_str() + t + 6, nullptr, 10);
  return true;
}

// "0-3,8,10-11" -> {0, 1, 2, 3, 8, 10, 11}
std::vector<uint32_t> cpu_list(const std::string& s) {
  std::vector<uint32_t> out;
  const char* p = s.c_str();
  while (*p) {
    while (*p == ' ' || *p == ',' || *p == '\t') ++p;
    if (*p < '0' || *p > '9') break;
    char* e = nullptr;
    const unsigned long a = std::strtoul(p, &e, 10);
    unsigned long b = a;
    p = e;
    if (*p == '-') b = std::strtoul(p + 1, &e, 10), p = e;
    for (unsigned long c = a; c <= b && c < 65536; ++c) out.push_back((uint32_t)c);
  }
  return out;
}

// Cpus_allowed_list of /proc/<pid>/status (empty: unreadable)
std::vector<uint32_t> allowed_cpus(const std::string& proc_root, uint32_t pid) {
  std::string st;
  if (!read_small(join(proc_root, std::to_string(pid) + "/status"), &st)) return {};
  const size_t k = st.find("Cpus_allowed_list:");
  if (k == std::string::npos) return {};
  const size_t e = st.find('\n', k);
  return cpu_list(st.substr(k + 18, (e == std::string::npos ? st.size() : e) - k - 18));
}

}  // namespace

// Busy jiffies per CPU from /proc/stat (user nice system idle iowait irq softirq steal ...: all
// but idle and iowait).
bool ProcSampler::read_cpu_busy(std::vector<uint64_t>* out) {
  out->clear();
  std::string st;
  if (!read_small(join(cfg_.proc_root, "stat"), &st)) return false;
  size_t pos = 0;
  while (pos < st.size()) {
    size_t e = st.find('\n', pos);
    if (e == std::string::npos) e = st.size();
    if (e - pos > 4 && st.compare(pos, 3, "cpu") == 0 && st[pos + 3] >= '0' && st[pos + 3] <= '9') {
      char* p = nullptr;
      const unsigned long cpu = std::strtoul(st.c_str() + pos + 3, &p, 10);
      uint64_t f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int i = 0; i < 8 && p < st.c_str() + e; ++i) f[i] = std::strtoull(p, &p, 10);
      if (cpu < 65536) {
        if (out->size() <= cpu) out->resize(cpu + 1, 0);
        (*out)[cpu] = f[0] + f[1] + f[2] + f[5] + f[6] + f[7];
      }
    }
    pos = e + 1;
  }
  return !out->empty();
}

ProcSampler::ProcSampler(Ring* ring, ProcSamplerConfig cfg) : ring_(ring), cfg_(std::move(cfg)) {}

ProcSampler::~ProcSampler() {
  stop();
  for (auto& kv : procs_) close_tasks(kv.second);
}

void ProcSampler::close_tasks(Proc& p) {
  for (auto& t : p.task_fds) ::close(t.second);
  p.task_fds.clear();
  p.listed = false;
}

// (Re-)list the process's threads: keep the open files of threads still there, open the new ones.
void ProcSampler::list_tasks(uint32_t pid, Proc& p, uint64_t mono_ns) {
  const std::string task = join(cfg_.proc_root, std::to_string(pid) + "/task");
  std::vector<uint32_t> tids;
  if (DIR* dir = ::opendir(task.c_str())) {
    while (dirent* de = ::readdir(dir)) {
      const char* n = de->d_name;
      if (*n < '0' || *n > '9') continue;
      tids.push_back((uint32_t)std::strtoul(n, nullptr, 10));
    }
    ::closedir(dir);
  }
  std::sort(tids.begin(), tids.end());
  std::vector<std::pair<uint32_t, int>> next;
  size_t j = 0;
  for (uint32_t tid : tids) {
    while (j < p.task_fds.size() && p.task_fds[j].first < tid) ::close(p.task_fds[j++].second);  // gone
    if (j < p.task_fds.size() && p.task_fds[j].first == tid) {
      next.push_back(p.task_fds[j++]);
      continue;
    }
    const int fd = ::open(join(task, std::to_string(tid) + "/schedstat").c_str(), O_RDONLY | O_CLOEXEC);
    if (fd >= 0) next.emplace_back(tid, fd);
  }
  for (; j < p.task_fds.size(); ++j) ::close(p.task_fds[j].second);
  p.task_fds.swap(next);
  p.listed_ns = mono_ns;
  p.listed = true;
}

void ProcSampler::set_targets(const std::vector<std::pair<uint32_t, uint32_t>>& pid_pod) {
  std::lock_guard<std::mutex> lk(mu_);
  targets_ = pid_pod;
}

// The process's cgroup files: the quota group's cpu.stat (nearest ancestor with a CFS quota),
// memory.pressure of its group (else the node's), cpu.pressure of its group (opt-in).
void ProcSampler::resolve(uint32_t pid, Proc& p) {
  p.resolved = true;
  p.ns_pid = ns_pid_of(cfg_.proc_root, pid);
  p.cpus = allowed_cpus(cfg_.proc_root, pid);
  std::string cg;
  if (!read_small(join(cfg_.proc_root, std::to_string(pid) + "/cgroup"), &cg)) return;
  const std::string root = cfg_.cgroup_root;
  size_t pos = 0;
  while (pos < cg.size()) {
    size_t e = cg.find('\n', pos);
    if (e == std::string::npos) e = cg.size();
    const std::string ln = cg.substr(pos, e - pos);
    pos = e + 1;
    const size_t c1 = ln.find(':');
    const size_t c2 = c1 == std::string::npos ? std::string::npos : ln.find(':', c1 + 1);
    if (c2 == std::string::npos) continue;
    const std::string ctrls = ln.substr(c1 + 1, c2 - c1 - 1), path = ln.substr(c2 + 1);
    if (ln.compare(0, c1, "0") == 0 && ctrls.empty()) {  // cgroup v2
      const std::string base = join(root, path);
      for (std::string d = base;; d = parent(d)) {
        std::string mx;
        if (read_small(join(d, "cpu.max"), &mx) && mx.compare(0, 3, "max") != 0 && !mx.empty()) {
          p.cfs_file = join(d, "cpu.stat");
          break;
        }
        if (d.size() <= root.size() || d == "/") break;
      }
      if (readable(join(base, "memory.pressure"))) p.mem_file = join(base, "memory.pressure");
      if (cfg_.cgroup_cpu_psi && readable(join(base, "cpu.pressure"))) p.cpu_psi_file = join(base, "cpu.pressure");
    } else if (p.cfs_file.empty()) {  // cgroup v1: the hierarchy holding the cpu controller
      bool cpu = false;
      for (size_t a = 0; a <= ctrls.size();) {
        size_t b = ctrls.find(',', a);
        if (b == std::string::npos) b = ctrls.size();
        if (ctrls.compare(a, b - a, "cpu") == 0) cpu = true;
        a = b + 1;
      }
      if (!cpu) continue;
      const std::string mnt = join(root, ctrls);
      for (std::string d = join(mnt, path);; d = parent(d)) {
        std::string q;
        if (read_small(join(d, "cpu.cfs_quota_us"), &q) && std::strtoll(q.c_str(), nullptr, 10) > 0) {
          p.cfs_file = join(d, "cpu.stat");
          break;
        }
        if (d.size() <= mnt.size() || d == "/") break;
      }
    }
  }
  if (p.mem_file.empty() && readable(join(cfg_.proc_root, "pressure/memory")))
    p.mem_file = join(cfg_.proc_root, "pressure/memory");
}

// This tick's growth of a group counter in ns: 0 on its first reading (it only primes) and when
// unreadable; read once per tick however many targets share the group.
uint64_t ProcSampler::group_delta(const std::string& file, int kind) {
  Group& g = groups_[file];
  if (g.seen) return g.delta;
  g.seen = true;
  g.delta = 0;
  std::string s;
  uint64_t v = 0, us = 0;
  bool got = false;
  if (read_small(file, &s)) {
    if (kind == 0) {
      if (keyed_u64(s, "throttled_usec", &us)) {
        v = us * 1000, got = true;
      } else if (keyed_u64(s, "throttled_time", &v)) {  // cgroup v1: ns
        got = true;
      }
    } else if (psi_some_us(s, &us)) {
      v = us * 1000, got = true;
    }
  }
  if (!got) return 0;
  if (g.have && v >= g.last) g.delta = v - g.last;
  g.have = true;
  g.last = v;
  return g.delta;
}

std::vector<EventRec> ProcSampler::tick(int64_t wall_ns, uint64_t mono_ns) {
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<EventRec> out;
  std::lock_guard<std::mutex> lk(mu_);
  const uint32_t mask = mask_.load(std::memory_order_relaxed);
  const uint64_t dt = prev_mono_ && mono_ns > prev_mono_ ? mono_ns - prev_mono_ : 0;
  prev_mono_ = mono_ns;
  for (auto& kv : groups_) kv.second.seen = false;
  std::map<std::pair<uint32_t, uint32_t>, Tid> next;
  std::map<uint32_t, Proc> live;
  uint64_t cfs_groups = 0;
  auto rec = [&](uint16_t type, uint32_t ns_pid, uint32_t pid, uint32_t pod, uint64_t value) {
    EventRec e{};
    e.ts_ns = wall_ns;
    e.value = value;
    e.pid = ns_pid;
    e.tid = pid;
    e.pod_id = pod;
    e.node_id = (uint16_t)cfg_.node_id;
    e.signal_type = type;
    out.push_back(e);
  };
  // pass 1: every watched process's threads (run-queue wait, on-CPU time)
  struct Obs {
    uint32_t pid, pod;
    uint64_t w_sum, s_sum, w_all, r_all;
  };
  std::vector<Obs> obs;
  for (const auto& tp : targets_) {
    const uint32_t pid = tp.first, pod = tp.second;
    if (live.count(pid)) continue;  // listed twice
    auto pit = procs_.find(pid);
    Proc pr = pit != procs_.end() ? pit->second : Proc{};
    if (pit != procs_.end()) pit->second.task_fds.clear();  // moved into pr
    if (!pr.listed || mono_ns < pr.listed_ns || mono_ns - pr.listed_ns >= task_rescan_ns_)
      list_tasks(pid, pr, mono_ns);
    if (pr.task_fds.empty()) {  // the process is gone (or unreadable)
      close_tasks(pr);
      continue;
    }
    uint64_t w_sum = 0, s_sum = 0, w_all = 0, r_all = 0;
    for (const auto& tf : pr.task_fds) {
      const uint32_t tid = tf.first;
      char buf[128];
      const ssize_t nr = ::pread(tf.second, buf, sizeof(buf) - 1, 0);
      if (nr <= 0) continue;  // the thread exited (dropped at the next listing)
      buf[nr] = 0;
      char* p = nullptr;
      const uint64_t run = std::strtoull(buf, &p, 10);
      const uint64_t wait = std::strtoull(p, &p, 10), slices = std::strtoull(p, &p, 10);
      const auto key = std::make_pair(pid, tid);
      next[key] = Tid{run, wait, slices};
      auto it = prev_.find(key);
      if (it == prev_.end()) continue;
      const uint64_t dw = wait >= it->second.wait ? wait - it->second.wait : 0;
      const uint64_t ds = slices >= it->second.slices ? slices - it->second.slices : 0;
      r_all += run >= it->second.run ? run - it->second.run : 0;
      w_all += dw;
      if (ds > 0 && dw >= cfg_.runq_floor_ns * ds) {  // this thread's waits reach the probe's floor
        w_sum += dw;
        s_sum += ds;
      }
    }
    if (!pr.resolved) resolve(pid, pr);
    live[pid] = pr;
    obs.push_back(Obs{pid, pod, w_sum, s_sum, w_all, r_all});
  }
  // each process's wait share this interval (milli-percent of one CPU; its group's cpu.pressure
  // share where that is larger)
  std::vector<uint64_t> milli(obs.size(), 0);
  for (size_t i = 0; i < obs.size(); ++i) {
    const Proc& pr = live[obs[i].pid];
    const uint64_t psi_d = pr.cpu_psi_file.empty() ? 0 : group_delta(pr.cpu_psi_file, 1);  // read every tick
    if (!dt) continue;
    milli[i] = (uint64_t)((double)obs[i].w_all * 100000.0 / (double)dt);
    const uint64_t m2 = (uint64_t)((double)psi_d * 100000.0 / (double)dt);
    if (m2 > milli[i]) milli[i] = m2;
  }
  // neighbours' load on the CPUs of each pod pinned to a small set: /proc/stat busy time of the set
  // less the pod's own on-CPU time, milli-percent of the set's capacity. Read only while such a pod
  // waits at the floor (on a large host /proc/stat costs ~1 ms of kernel time per read), so the
  // first interval at the floor has no delta yet and counts as unconfirmed (-2); -1: not gated.
  std::map<uint32_t, int64_t> foreign;
  if (cfg_.steal_foreign_milli && (mask >> kSigSteal & 1)) {
    std::map<uint32_t, std::pair<std::vector<bool>, uint64_t>> pods;  // pod -> (CPU set, on-CPU ns)
    std::map<uint32_t, bool> unknown;
    for (const Obs& o : obs) {
      const Proc& pr = live[o.pid];
      auto& e = pods[o.pod];
      if (pr.cpus.empty()) unknown[o.pod] = true;
      for (uint32_t c : pr.cpus) {
        if (e.first.size() <= c) e.first.resize(c + 1, false);
        e.first[c] = true;
      }
      e.second += o.r_all;
    }
    bool need = false;
    for (const auto& kv : pods) {
      const uint64_t n = (uint64_t)std::count(kv.second.first.begin(), kv.second.first.end(), true);
      foreign[kv.first] = (unknown.count(kv.first) || n == 0 || n > cfg_.steal_foreign_max_cpus) ? -1 : -2;
    }
    for (size_t i = 0; i < obs.size(); ++i)
      if (milli[i] >= cfg_.steal_floor_milli && foreign[obs[i].pod] == -2) need = true;
    if (need) {
      std::vector<uint64_t> busy;
      const bool have = read_cpu_busy(&busy);
      const bool valid = have && cpu_busy_have_ && cpu_busy_tick_ + 1 == st_.ticks && dt;
      const double ns_per_jiffy = 1e9 / (double)std::max(1L, ::sysconf(_SC_CLK_TCK));
      for (const auto& kv : pods) {
        if (foreign[kv.first] != -2 || !valid) continue;
        uint64_t n = 0, jif = 0;
        bool ok = true;
        for (size_t c = 0; c < kv.second.first.size(); ++c) {
          if (!kv.second.first[c]) continue;
          ++n;
          if (c >= busy.size() || c >= cpu_busy_.size()) {
            ok = false;
            break;
          }
          jif += busy[c] >= cpu_busy_[c] ? busy[c] - cpu_busy_[c] : 0;
        }
        if (!ok) continue;  // a CPU missing from /proc/stat: unconfirmed
        const double busy_ns = (double)jif * ns_per_jiffy, own = (double)kv.second.second;
        const double f = busy_ns > own ? busy_ns - own : 0.0;
        foreign[kv.first] = (int64_t)(f * 100000.0 / ((double)dt * (double)n));
      }
      cpu_busy_.swap(busy);
      cpu_busy_have_ = have;
      cpu_busy_tick_ = st_.ticks;
    } else {
      cpu_busy_have_ = false;
    }
  }
  // pass 2: the records, per process in watch order
  for (const Obs& o : obs) {
    const uint32_t pid = o.pid, pod = o.pod;
    Proc& pr = live[pid];
    if ((mask >> kSigRunq & 1) && o.s_sum && o.w_sum / o.s_sum >= cfg_.runq_floor_ns)
      rec(kSigRunq, pr.ns_pid, pid, pod, o.w_sum / o.s_sum);
    if ((mask >> kSigSteal & 1) && dt) {
      const uint64_t m = milli[&o - obs.data()];
      bool at_floor = m >= cfg_.steal_floor_milli;
      const auto fit = foreign.find(pod);
      if (at_floor && fit != foreign.end() && fit->second != -1 &&
          (fit->second == -2 || (uint64_t)fit->second < cfg_.steal_foreign_milli)) {
        at_floor = false;  // the pod waited behind its own threads: no neighbour held its CPUs
        ++st_.steal_gated;
      }
      pr.steal_run = at_floor ? pr.steal_run + 1 : 0;
      if (pr.steal_run >= std::max<uint32_t>(1, cfg_.steal_sustain)) rec(kSigSteal, pr.ns_pid, pid, pod, m);
    }
    if (!pr.cfs_file.empty()) {
      ++cfs_groups;
      const uint64_t d = group_delta(pr.cfs_file, 0);
      if ((mask >> kSigCfs & 1) && d >= cfg_.cfs_floor_ns) rec(kSigCfs, pr.ns_pid, pid, pod, d);
    }
    if (!pr.mem_file.empty()) {
      const uint64_t d = group_delta(pr.mem_file, 1);
      if ((mask >> kSigMem & 1) && d >= cfg_.mem_floor_ns) rec(kSigMem, pr.ns_pid, pid, pod, d);
    }
  }
  prev_.swap(next);
  for (auto& kv : procs_) close_tasks(kv.second);  // processes no longer watched (the rest moved)
  procs_.swap(live);
  for (auto it = groups_.begin(); it != groups_.end();) it = it->second.seen ? std::next(it) : groups_.erase(it);
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
  }
  ++st_.ticks;
  st_.targets = targets_.size();
  st_.cfs_groups = cfs_groups;
  if (ring_) {
    st_.emitted += pushed;
    st_.dropped += out.size() - pushed;
  } else {
    st_.emitted += out.size();
  }
  for (const EventRec& e : out)
    ++st_.by_type[e.signal_type == kSigRunq ? 0 : e.signal_type == kSigSteal ? 1 : e.signal_type == kSigMem ? 2 : 3];
  const uint64_t took = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now() - t0).count();
  st_.last_tick_ns = took;
  if (took > st_.max_tick_ns) st_.max_tick_ns = took;
  return out;
}

void ProcSampler::start(uint64_t interval_ns) {
  stop();
  {
    std::lock_guard<std::mutex> lk(tmu_);
    stop_ = false;
  }
  thr_ = std::thread([this, interval_ns] {
    std::unique_lock<std::mutex> lk(tmu_);
    while (!cv_.wait_for(lk, std::chrono::nanoseconds(interval_ns), [this] { return stop_; })) {
      if (paused_.load(std::memory_order_relaxed)) continue;
      lk.unlock();
      timespec rt{}, mo{};
      clock_gettime(CLOCK_REALTIME, &rt);
      clock_gettime(CLOCK_MONOTONIC, &mo);
      tick((int64_t)rt.tv_sec * 1000000000ll + rt.tv_nsec, (uint64_t)mo.tv_sec * 1000000000ull + (uint64_t)mo.tv_nsec);
      lk.lock();
    }
  });
}

void ProcSampler::stop() {
  {
    std::lock_guard<std::mutex> lk(tmu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (thr_.joinable()) thr_.join();
}

ProcSamplerStats ProcSampler::stats() {
  std::lock_guard<std::mutex> lk(mu_);
  return st_;
}

}  // namespace mislo
