"""Unprivileged kernel signals from /proc: the agent's own producer where BPF is not allowed.

REF's min-capability mode keeps two signals (dns, tcp) and drops the scheduler ones with the BPF
programs (/root/reference/docs/security/agent-min-capability-mode.md:1-35). The scheduler already
accounts what ``runqueue_delay.bpf.c`` measures: ``/proc/<pid>/task/<tid>/schedstat`` holds each
thread's on-CPU time, run-queue wait time and timeslice count, readable without privilege. The
``SchedstatSampler`` turns their per-interval deltas into ``runqueue_delay_ms`` records -- per
process, the run-queue wait over the timeslices of its threads whose mean wait per timeslice
reached the probe's 100 us floor (each timeslice is one wakeup-to-run the BPF probe times, and
the probe emits only waits above its floor, so this is the mean of the waits the probe would
have emitted for the process; without the filter the many near-zero waits of a runtime's
helper threads hid a starved main thread: config-3 run, profiles/r3_config3_*) -- tagged with
the pid and pod, and pushes
them into the agent's user-space ring like the rocprofiler tool's records. The GPU window engine
joins them to the pod's spans (pod + pid tier).

Memory: the pressure-stall accounting (PSI, ``memory.pressure`` of the process's cgroup v2, else
the node's ``/proc/pressure/memory``) says how long tasks stalled on memory -- reclaim, refaults,
swap-in -- in every interval. Its per-interval growth becomes ``mem_reclaim_latency_ms`` records
(the reclaim probe's signal) for the watched processes, so memory pressure is observed, not
assumed absent, by an agent without BPF.

Watched processes: a static ``pid -> pod uid`` list (``agent --procfs-pods``), or every process in
the node's kubepods cgroups (``pod_processes``). They are named by the agent's (host) pids; the
records carry each process's pid in its own innermost pid namespace (``/proc/<pid>/status``
NSpid), the pid its spans and its rocprofiler records carry, as the BPF probes do
(mislo_probe.h mislo_ns_tgid).
"""

from __future__ import annotations

import os
import threading
import time
from typing import Callable, Dict, Iterable, List, Optional, Tuple

import numpy as np

from . import records

RUNQUEUE_TYPE = 3          # catalogue kernel type of runqueue_delay_ms (ns in the record)
MEM_RECLAIM_TYPE = 7       # catalogue kernel type of mem_reclaim_latency_ms (ns in the record)
FLOOR_NS = 100_000         # runqueue_delay.bpf.c's emit floor


def psi_path(pid: int, proc_root: str = "/proc", cgroup_root: str = "/sys/fs/cgroup") -> Optional[str]:
    """The memory.pressure file covering ``pid``: its cgroup v2 group's, else the node's."""
    try:
        with open(os.path.join(proc_root, str(pid), "cgroup")) as fh:
            for ln in fh:
                if ln.startswith("0::"):
                    p = os.path.join(cgroup_root, ln[3:].strip().lstrip("/"), "memory.pressure")
                    if os.access(p, os.R_OK):
                        return p
    except OSError:
        pass
    p = os.path.join(proc_root, "pressure", "memory")
    return p if os.access(p, os.R_OK) else None


def read_psi_total_us(path: str) -> Optional[int]:
    """``some ... total=<us>`` of a PSI file."""
    try:
        with open(path) as fh:
            for ln in fh:
                if ln.startswith("some"):
                    return int(ln.rsplit("total=", 1)[1])
    except (OSError, ValueError, IndexError):
        return None
    return None


def psi_available(proc_root: str = "/proc") -> bool:
    return read_psi_total_us(os.path.join(proc_root, "pressure", "memory")) is not None


def ns_pid(pid: int, proc_root: str = "/proc") -> int:
    """``pid``'s pid in its innermost pid namespace (the last NSpid field; ``pid`` itself for a
    process in the reader's namespace or when the field is unavailable)."""
    try:
        with open(os.path.join(proc_root, str(pid), "status")) as fh:
            for ln in fh:
                if ln.startswith("NSpid:"):
                    f = ln.split()
                    return int(f[-1]) if len(f) > 1 else pid
    except (OSError, ValueError):
        pass
    return pid


def read_schedstat(path: str) -> Optional[Tuple[int, int, int]]:
    try:
        with open(path) as fh:
            f = fh.read().split()
        return int(f[0]), int(f[1]), int(f[2])
    except (OSError, ValueError, IndexError):
        return None


STEAL_TYPE = 6             # catalogue kernel type of cpu_steal_pct (milli-percent in the record)
CFS_TYPE = 12              # catalogue kernel type of cfs_throttled_ms (ns in the record)
# 20 % of one CPU over the interval: a healthy multi-threaded service's own threads contend for
# its CPUs at a few percent (config-3 baseline on MI355X: 27 of ~150 intervals of the RAG service
# at 2-8 %, 7 above 8 %; under the CPU fault every interval well above 8 %, profiles/r4_config3_first)
STEAL_FLOOR_MILLI = 20000
# ... held for this many consecutive intervals: the healthy service's threads still crossed 20 % in
# ~1 of 30 intervals, one at a time (5 cpu_throttle false positives in 15 baseline windows,
# profiles/r4_config3_gated), while a starved service stays above it in every interval
STEAL_SUSTAIN = 3
# ... and, for a pod on a small CPU set (at most STEAL_FOREIGN_MAX_CPUS), only while other processes
# kept at least this share of those CPUs busy: after a CPU fault a pod working off its backlog waits
# behind its own threads (6 of 8 recovery windows read cpu_throttle in one config-3 run,
# profiles/r4_config3_rerun)
STEAL_FOREIGN_MILLI = 25000
STEAL_FOREIGN_MAX_CPUS = 32
SIGNAL_TYPES = {"runqueue_delay_ms": RUNQUEUE_TYPE, "cpu_steal_pct": STEAL_TYPE,
                "mem_reclaim_latency_ms": MEM_RECLAIM_TYPE, "cfs_throttled_ms": CFS_TYPE}
ALL_MASK = sum(1 << t for t in SIGNAL_TYPES.values())


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as fh:
            return fh.read()
    except OSError:
        return None


def cpu_list(text: str) -> List[int]:
    """"0-3,8,10-11" -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in text.replace(" ", "").split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        try:
            lo = int(a)
            hi = int(b) if b else lo
        except ValueError:
            break
        out.extend(range(lo, min(hi, 65535) + 1))
    return out


def allowed_cpus(pid: int, proc_root: str = "/proc") -> List[int]:
    """Cpus_allowed_list of /proc/<pid>/status ([] = unreadable)."""
    text = _read(os.path.join(proc_root, str(pid), "status")) or ""
    for ln in text.splitlines():
        if ln.startswith("Cpus_allowed_list:"):
            return cpu_list(ln.split(":", 1)[1].strip())
    return []


def cpu_busy_jiffies(proc_root: str = "/proc") -> Dict[int, int]:
    """Busy jiffies per CPU from /proc/stat: every field but idle and iowait."""
    out: Dict[int, int] = {}
    for ln in (_read(os.path.join(proc_root, "stat")) or "").splitlines():
        if ln.startswith("cpu") and len(ln) > 3 and ln[3].isdigit():
            f = ln.split()
            try:
                v = [int(x) for x in f[1:9]] + [0] * 8
            except ValueError:
                continue
            out[int(f[0][3:])] = v[0] + v[1] + v[2] + v[5] + v[6] + v[7]
    return out


def cgroup_files(pid: int, proc_root: str = "/proc", cgroup_root: str = "/sys/fs/cgroup",
                 cpu_psi: bool = False) -> Tuple[str, str, str]:
    """(quota group's cpu.stat, memory PSI file, cpu PSI file) of ``pid`` ("" = none):
    runtime/csrc/procsampler.cpp ProcSampler::resolve. The CFS throttling of a process is its
    nearest ancestor group with a CPU quota (cgroup v2 cpu.max, v1 cpu.cfs_quota_us)."""
    cfs = mem = cpu = ""
    text = _read(os.path.join(proc_root, str(pid), "cgroup"))
    root = cgroup_root.rstrip("/")
    for ln in (text or "").splitlines():
        parts = ln.split(":", 2)
        if len(parts) != 3:
            continue
        hid, ctrls, path = parts
        if hid == "0" and not ctrls:  # v2
            base = os.path.join(root, path.lstrip("/")).rstrip("/") or "/"
            d = base
            while True:
                mx = _read(os.path.join(d, "cpu.max"))
                if mx and not mx.startswith("max"):
                    cfs = os.path.join(d, "cpu.stat")
                    break
                if len(d) <= len(root) or d == "/":
                    break
                d = os.path.dirname(d)
            if os.access(os.path.join(base, "memory.pressure"), os.R_OK):
                mem = os.path.join(base, "memory.pressure")
            if cpu_psi and os.access(os.path.join(base, "cpu.pressure"), os.R_OK):
                cpu = os.path.join(base, "cpu.pressure")
        elif not cfs and "cpu" in ctrls.split(","):  # v1
            mnt = os.path.join(root, ctrls)
            d = os.path.join(mnt, path.lstrip("/")).rstrip("/")
            while True:
                q = _read(os.path.join(d, "cpu.cfs_quota_us"))
                try:
                    if q is not None and int(q.strip()) > 0:
                        cfs = os.path.join(d, "cpu.stat")
                        break
                except ValueError:
                    pass
                if len(d) <= len(mnt) or d == "/":
                    break
                d = os.path.dirname(d)
    if not mem and os.access(os.path.join(proc_root, "pressure", "memory"), os.R_OK):
        mem = os.path.join(proc_root, "pressure", "memory")
    return cfs, mem, cpu


def read_throttled_ns(path: str) -> Optional[int]:
    """cpu.stat throttled_usec (v2, -> ns) or throttled_time (v1, ns)."""
    text = _read(path)
    if text is None:
        return None
    kv = dict(ln.split(" ", 1) for ln in text.splitlines() if " " in ln)
    try:
        if "throttled_usec" in kv:
            return int(kv["throttled_usec"]) * 1000
        if "throttled_time" in kv:
            return int(kv["throttled_time"])
    except ValueError:
        return None
    return None


class SchedstatSampler:
    """The Python model of the native sampler (runtime/csrc/procsampler.cpp, ``NativeSampler``):
    per watched process and interval, in this order,

    * ``runqueue_delay_ms``: the mean run-queue wait per timeslice over its threads whose mean
      reached the probe's 100 us floor;
    * ``cpu_steal_pct``: its threads' summed run-queue wait over the interval, in percent of one
      CPU (milli-percent in the record) -- CPU the process wanted and did not get; with
      ``cpu_psi`` the larger of that and its (pod-private) group's cpu.pressure "some" share;
    * ``cfs_throttled_ms``: the growth of its quota group's throttled time (CFS bandwidth);
    * ``mem_reclaim_latency_ms``: the growth of its group's PSI memory stall (else the node's).

    The agent runs the native sampler; this class is its oracle in the tests and the fallback
    where the native runtime is not built."""

    def __init__(self, targets: Callable[[], Dict[int, int]], push: Callable[[np.ndarray], int], rec: int = 24,
                 proc_root: str = "/proc", floor_ns: int = FLOOR_NS, node_id: int = 0,
                 cgroup_root: str = "/sys/fs/cgroup", cpu_psi: bool = False,
                 steal_floor_milli: int = STEAL_FLOOR_MILLI, steal_sustain: int = STEAL_SUSTAIN,
                 steal_foreign_milli: int = STEAL_FOREIGN_MILLI, steal_foreign_max_cpus: int = STEAL_FOREIGN_MAX_CPUS):
        """``targets()`` -> {pid: pod id}; ``push(records)`` -> records accepted (the user ring)."""
        self.targets, self.push, self.rec = targets, push, int(rec)
        self.proc_root, self.floor_ns, self.node_id = proc_root, int(floor_ns), int(node_id)
        self.cgroup_root, self.cpu_psi, self.steal_floor = cgroup_root, bool(cpu_psi), int(steal_floor_milli)
        self.steal_sustain = max(1, int(steal_sustain))
        self.steal_foreign, self.steal_foreign_max_cpus = int(steal_foreign_milli), int(steal_foreign_max_cpus)
        self._cpu_busy: Optional[Dict[int, int]] = None
        self._cpu_busy_tick = -1
        self.steal_gated = 0
        self._steal_run: Dict[int, int] = {}  # pid -> consecutive intervals at the floor
        self.mask = ALL_MASK
        self.paused = False
        self._prev: Dict[Tuple[int, int], Tuple[int, int, int]] = {}  # (pid, tid) -> (run, wait, slices)
        self._procs: Dict[int, tuple] = {}  # pid -> (ns pid, cfs, mem, cpu psi files, allowed CPUs)
        self._groups: Dict[str, int] = {}                      # file -> last reading (ns)
        self._prev_mono: Optional[int] = None
        self.samples = self.emitted = self.dropped = 0
        self._stop = threading.Event()
        self._thr: Optional[threading.Thread] = None

    def _group_delta(self, path: str, kind: int, cache: Dict[str, int]) -> int:
        if path in cache:
            return cache[path]
        v = read_throttled_ns(path) if kind == 0 else read_psi_total_us(path)
        d = 0
        if v is not None:
            v = v if kind == 0 else v * 1000
            last = self._groups.get(path)
            if last is not None and v >= last:
                d = v - last
            self._groups[path] = v
        cache[path] = d
        return d

    def sample(self, now_ns: Optional[int] = None, mono_ns: Optional[int] = None) -> np.ndarray:
        """One interval: EVENT records of the watched processes (see the class docstring)."""
        now = int(now_ns if now_ns is not None else time.time_ns())
        # an interval given only as wall-clock times (tests) is measured on that clock
        mono = int(mono_ns if mono_ns is not None else (now if now_ns is not None else time.monotonic_ns()))
        dt = mono - self._prev_mono if self._prev_mono is not None and mono > self._prev_mono else 0
        self._prev_mono = mono
        rows = []
        nxt: Dict[Tuple[int, int], Tuple[int, int, int]] = {}
        live: Dict[int, tuple] = {}
        cache: Dict[str, int] = {}
        obs = []  # pass 1: (pid, pod, w_sum, s_sum, w_all, r_all)
        for pid, pod in self.targets().items():
            task = os.path.join(self.proc_root, str(pid), "task")
            try:
                tids = sorted(int(t) for t in os.listdir(task) if t.isdigit())
            except OSError:
                continue
            w_sum = s_sum = w_all = r_all = 0
            for tid in tids:
                st = read_schedstat(os.path.join(task, str(tid), "schedstat"))
                if st is None:
                    continue
                key = (pid, tid)
                nxt[key] = (st[0], st[1], st[2])
                prev = self._prev.get(key)
                if prev is None:
                    continue
                dr, dw, ds = max(0, st[0] - prev[0]), max(0, st[1] - prev[1]), max(0, st[2] - prev[2])
                r_all += dr
                w_all += dw
                if ds > 0 and dw >= self.floor_ns * ds:  # this thread's waits reach the floor
                    w_sum += dw
                    s_sum += ds
            info = self._procs.get(pid)
            if info is None:
                info = ((ns_pid(pid, self.proc_root),) + cgroup_files(pid, self.proc_root, self.cgroup_root, self.cpu_psi)
                        + (allowed_cpus(pid, self.proc_root),))
            live[pid] = info
            obs.append((pid, pod, w_sum, s_sum, w_all, r_all))
        milli = []  # each process's wait share (milli-percent of one CPU; its cpu.pressure share if larger)
        for pid, pod, _, _, w_all, _ in obs:
            cpu = live[pid][3]
            psi_d = self._group_delta(cpu, 1, cache) if cpu else 0  # read every tick
            milli.append(max(int(float(w_all) * 100000.0 / float(dt)), int(float(psi_d) * 100000.0 / float(dt)))
                         if dt else 0)
        # neighbours' load on the CPUs of each pod pinned to a small set (runtime/csrc/procsampler.cpp
        # tick): /proc/stat busy time of the set less the pod's own on-CPU time, milli-percent of the
        # set's capacity; read only while such a pod waits at the floor (-2: no delta yet, unconfirmed;
        # -1: not gated)
        foreign: Dict[int, int] = {}
        if self.steal_foreign and self.mask >> STEAL_TYPE & 1:
            sets: Dict[int, set] = {}
            own: Dict[int, int] = {}
            unknown = set()
            for pid, pod, _, _, _, r_all in obs:
                cpus = live[pid][4]
                if not cpus:
                    unknown.add(pod)
                sets.setdefault(pod, set()).update(cpus)
                own[pod] = own.get(pod, 0) + r_all
            for pod, cs in sets.items():
                foreign[pod] = -1 if pod in unknown or not cs or len(cs) > self.steal_foreign_max_cpus else -2
            need = any(m >= self.steal_floor and foreign[o[1]] == -2 for m, o in zip(milli, obs))
            if need:
                busy = cpu_busy_jiffies(self.proc_root)
                valid = bool(busy) and self._cpu_busy is not None and self._cpu_busy_tick + 1 == self.samples and dt > 0
                ns_per_jiffy = 1e9 / float(max(1, os.sysconf("SC_CLK_TCK")))
                for pod, cs in sets.items():
                    if foreign[pod] != -2 or not valid or not all(c in busy and c in self._cpu_busy for c in cs):
                        continue
                    jif = sum(max(0, busy[c] - self._cpu_busy[c]) for c in cs)
                    f = max(0.0, float(jif) * ns_per_jiffy - float(own[pod]))
                    foreign[pod] = int(f * 100000.0 / (float(dt) * float(len(cs))))
                self._cpu_busy = busy or None
                self._cpu_busy_tick = self.samples
            else:
                self._cpu_busy = None
        for i, (pid, pod, w_sum, s_sum, w_all, _) in enumerate(obs):  # pass 2: the records, in watch order
            npid, cfs, mem, cpu, _ = live[pid]
            if self.mask >> RUNQUEUE_TYPE & 1 and s_sum and w_sum // s_sum >= self.floor_ns:
                rows.append((RUNQUEUE_TYPE, npid, pid, pod, w_sum // s_sum))
            if self.mask >> STEAL_TYPE & 1 and dt:
                m = milli[i]
                at_floor = m >= self.steal_floor
                fg = foreign.get(pod, -1)
                if at_floor and fg != -1 and (fg == -2 or fg < self.steal_foreign):
                    at_floor = False  # the pod waited behind its own threads: no neighbour held its CPUs
                    self.steal_gated += 1
                run = self._steal_run.get(pid, 0) + 1 if at_floor else 0
                self._steal_run[pid] = run
                if run >= self.steal_sustain:
                    rows.append((STEAL_TYPE, npid, pid, pod, m))
            if cfs:
                d = self._group_delta(cfs, 0, cache)
                if self.mask >> CFS_TYPE & 1 and d >= self.floor_ns:
                    rows.append((CFS_TYPE, npid, pid, pod, d))
            if mem:
                d = self._group_delta(mem, 1, cache)
                if self.mask >> MEM_RECLAIM_TYPE & 1 and d >= self.floor_ns:
                    rows.append((MEM_RECLAIM_TYPE, npid, pid, pod, d))
        self._prev = nxt
        self._procs = live
        self._steal_run = {p: r for p, r in self._steal_run.items() if p in live}
        self._groups = {k: v for k, v in self._groups.items() if k in cache}
        self.samples += 1
        ev = np.zeros(len(rows), dtype=records.EVENT)
        if rows:
            a = np.array(rows, dtype=np.int64)
            ev["ts_ns"] = now
            ev["signal_type"] = a[:, 0].astype(np.uint16)
            ev["value"] = a[:, 4].astype(np.uint64)
            ev["pid"] = a[:, 1].astype(np.uint32)
            ev["tid"] = a[:, 2].astype(np.uint32)
            ev["pod_id"] = a[:, 3].astype(np.uint32)
            ev["node_id"] = self.node_id
        return ev

    def tick(self, now_ns: Optional[int] = None, mono_ns: Optional[int] = None) -> int:
        ev = self.sample(now_ns, mono_ns)
        if not len(ev):
            return 0
        n = int(self.push(records.to_user(ev, self.rec)))
        self.emitted += n
        self.dropped += len(ev) - n
        return n

    def start(self, interval_s: float = 0.1) -> "SchedstatSampler":
        def run():
            while not self._stop.wait(interval_s):
                if self.paused:
                    continue
                try:
                    self.tick()
                except Exception:  # noqa: BLE001 - a sampler hiccup must not stop the agent
                    self.dropped += 1

        self._thr = threading.Thread(target=run, name="procfs-sampler", daemon=True)
        self._thr.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thr is not None:
            self._thr.join(5)

    def stats(self) -> Dict[str, int]:
        return {"ticks": self.samples, "emitted": self.emitted, "dropped": self.dropped}


class NativeSampler:
    """The agent's sampler: runtime/csrc/procsampler.cpp on its own thread, pushing straight into
    the user ring (no Python per record or per file). ``targets`` is re-read every
    ``refresh_s`` by a light Python timer (pod churn); everything per interval is native."""

    def __init__(self, ring, targets: Callable[[], Dict[int, int]], node_id: int = 0, proc_root: str = "/proc",
                 cgroup_root: str = "/sys/fs/cgroup", cpu_psi: bool = False, floor_ns: int = FLOOR_NS,
                 steal_floor_milli: int = STEAL_FLOOR_MILLI, refresh_s: float = 10.0,
                 steal_sustain: int = STEAL_SUSTAIN, steal_foreign_milli: int = STEAL_FOREIGN_MILLI,
                 steal_foreign_max_cpus: int = STEAL_FOREIGN_MAX_CPUS):
        from ..runtime import load

        rt = load()
        self.targets, self.refresh_s = targets, float(refresh_s)
        self.native = rt.ProcSampler(ring, node_id, proc_root, cgroup_root, bool(cpu_psi), int(floor_ns),
                                     int(steal_floor_milli), int(floor_ns), int(floor_ns), int(steal_sustain),
                                     int(steal_foreign_milli), int(steal_foreign_max_cpus))
        self._stop = threading.Event()
        self._thr: Optional[threading.Thread] = None

    @property
    def mask(self) -> int:
        return int(self.native.mask)

    @mask.setter
    def mask(self, m: int) -> None:
        self.native.mask = int(m)

    @property
    def paused(self) -> bool:
        return bool(self.native.paused)

    @paused.setter
    def paused(self, p: bool) -> None:
        self.native.paused = bool(p)

    def refresh(self) -> None:
        self.native.set_target_list(sorted((int(p), int(v)) for p, v in self.targets().items()))

    def sample(self, now_ns: int, mono_ns: int) -> np.ndarray:
        """One interval by hand (tests): the EVENT records it produced (also pushed)."""
        return np.frombuffer(self.native.tick(int(now_ns), int(mono_ns)), dtype=records.EVENT)

    def start(self, interval_s: float = 0.1) -> "NativeSampler":
        self.refresh()
        self.native.start(float(interval_s))

        def run():
            while not self._stop.wait(self.refresh_s):
                try:
                    self.refresh()
                except Exception:  # noqa: BLE001 - keep the last target list
                    pass

        self._thr = threading.Thread(target=run, name="procfs-targets", daemon=True)
        self._thr.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        self.native.stop()
        if self._thr is not None:
            self._thr.join(5)

    def stats(self) -> Dict[str, int]:
        return dict(self.native.stats())


def parse_pod_list(spec: str) -> Dict[int, str]:
    """'pid:uid,pid:uid' -> {pid: uid}."""
    out: Dict[int, str] = {}
    for item in (spec or "").split(","):
        if ":" in item:
            pid, uid = item.split(":", 1)
            out[int(pid)] = uid.strip()
    return out


def pod_processes(cgroup_root: str = "/sys/fs/cgroup") -> Dict[int, str]:
    """{pid: pod uid} of every process in the node's kubepods cgroups."""
    from .bpf import _pod_uid

    out: Dict[int, str] = {}
    for dirpath, _dirs, files in os.walk(cgroup_root):
        if "cgroup.procs" not in files or "pod" not in dirpath:
            continue
        uid = ""
        for part in reversed(dirpath.split(os.sep)):
            uid = _pod_uid(part)
            if uid:
                break
        if not uid:
            continue
        try:
            with open(os.path.join(dirpath, "cgroup.procs")) as fh:
                for ln in fh:
                    if ln.strip().isdigit():
                        out[int(ln)] = uid
        except OSError:
            continue
    return out


class MultiSampler:
    """Several samplers as one (split rings: one per worker ring set); the shedding ladder sets
    the mask / pause on all of them."""

    def __init__(self, samplers):
        self.samplers = list(samplers)

    @property
    def mask(self) -> int:
        return max((s.mask for s in self.samplers), default=0)  # (KFD samplers report 0)

    @mask.setter
    def mask(self, m: int) -> None:
        for s in self.samplers:
            s.mask = m

    @property
    def paused(self) -> bool:
        return all(s.paused for s in self.samplers)

    @paused.setter
    def paused(self, p: bool) -> None:
        for s in self.samplers:
            s.paused = p

    def start(self, interval_s: float = 0.1) -> "MultiSampler":
        for s in self.samplers:
            s.start(interval_s)
        return self

    def stop(self) -> None:
        for s in self.samplers:
            s.stop()

    def stats(self) -> Dict[str, int]:
        out: Dict[str, int] = {}
        for s in self.samplers:
            for k, v in s.stats().items():
                out[k] = max(out.get(k, 0), v) if k in ("max_tick_ns", "last_tick_ns") else out.get(k, 0) + v
        return out


def local_addresses(pid: int, proc_root: str = "/proc") -> set:
    """The IPv4 addresses local to ``pid``'s network namespace (``/proc/<pid>/net/fib_trie``
    "/32 host LOCAL" entries), loopback excluded."""
    text = _read(os.path.join(proc_root, str(pid), "net", "fib_trie")) or ""
    out, last = set(), ""
    for ln in text.splitlines():
        t = ln.strip()
        if t.startswith("|--"):
            last = t[3:].strip()
        elif t.startswith("/32 host LOCAL") and last and not last.startswith("127."):
            out.add(last)
    return out


def pod_addresses(procs: Dict[int, str], proc_root: str = "/proc") -> Dict[str, set]:
    """{IP: pod uids} of the node's pods, from one process per pod (``procs``: pid -> pod uid, e.g.
    ``pod_processes()``): the OTLP receiver keeps a span that names a pod only when it arrives
    from that pod's address (collector/otlp.py SpanMapper)."""
    seen: Dict[str, int] = {}
    for pid, uid in sorted(procs.items()):
        seen.setdefault(uid, pid)
    out: Dict[str, set] = {}
    for uid, pid in seen.items():
        for ip in local_addresses(pid, proc_root):
            out.setdefault(ip, set()).add(uid)
    return out
