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
from typing import Callable, Dict, Iterable, Optional, Tuple

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


class SchedstatSampler:
    def __init__(self, targets: Callable[[], Dict[int, int]], push: Callable[[np.ndarray], int], rec: int = 24,
                 proc_root: str = "/proc", floor_ns: int = FLOOR_NS, node_id: int = 0):
        """``targets()`` -> {pid: pod id}; ``push(records)`` -> records accepted (the user ring)."""
        self.targets, self.push, self.rec = targets, push, int(rec)
        self.proc_root, self.floor_ns, self.node_id = proc_root, int(floor_ns), int(node_id)
        self._prev: Dict[Tuple[int, int], Tuple[int, int]] = {}
        self._psi: Dict[int, Tuple[Optional[str], Optional[int]]] = {}   # pid -> (PSI file, last total us)
        self._ns: Dict[int, int] = {}      # host pid -> pid in its own namespace
        self.samples = self.emitted = self.dropped = 0
        self._stop = threading.Event()
        self._thr: Optional[threading.Thread] = None

    def sample(self, now_ns: Optional[int] = None) -> np.ndarray:
        """One interval: EVENT records of the processes whose mean wait per timeslice crossed the floor."""
        now = int(now_ns if now_ns is not None else time.time_ns())
        rows, seen = [], set()
        for pid, pod in self.targets().items():
            task = os.path.join(self.proc_root, str(pid), "task")
            try:
                tids = [int(t) for t in os.listdir(task) if t.isdigit()]
            except OSError:
                continue
            w_sum = s_sum = 0
            for tid in tids:
                st = read_schedstat(os.path.join(task, str(tid), "schedstat"))
                if st is None:
                    continue
                key = (pid, tid)
                seen.add(key)
                prev = self._prev.get(key)
                self._prev[key] = (st[1], st[2])
                if prev is None:
                    continue
                dw, ds = st[1] - prev[0], st[2] - prev[1]
                if ds > 0 and dw >= self.floor_ns * ds:  # this thread's waits reach the floor
                    w_sum += dw
                    s_sum += ds
            if s_sum and w_sum // s_sum >= self.floor_ns:
                rows.append((self.pod_pid(pid), pid, pod, w_sum // s_sum))
        for key in list(self._prev):
            if key not in seen:
                del self._prev[key]
        alive = {k[0] for k in seen}
        for pid in list(self._ns):
            if pid not in alive:
                del self._ns[pid]
        mem = self._memory_rows()
        self.samples += 1
        ev = np.zeros(len(rows) + len(mem), dtype=records.EVENT)
        if len(ev):
            a = np.array(rows + mem, dtype=np.int64)
            ev["ts_ns"] = now
            ev["signal_type"] = np.where(np.arange(len(ev)) < len(rows), RUNQUEUE_TYPE, MEM_RECLAIM_TYPE)
            ev["value"] = a[:, 3].astype(np.uint64)
            ev["pid"] = a[:, 0].astype(np.uint32)
            ev["tid"] = a[:, 1].astype(np.uint32)
            ev["pod_id"] = a[:, 2].astype(np.uint32)
            ev["node_id"] = self.node_id
        return ev

    def pod_pid(self, pid: int) -> int:
        """The record's pid: ``pid`` as its own pod sees it (cached while it lives)."""
        v = self._ns.get(pid)
        if v is None:
            v = self._ns[pid] = ns_pid(pid, self.proc_root)
        return v

    def _memory_rows(self):
        """(pid, pid, pod, stall ns) of the watched processes whose PSI memory stall grew by at
        least the floor since the last interval."""
        rows = []
        live = set()
        totals: Dict[str, Optional[int]] = {}
        for pid, pod in self.targets().items():
            live.add(pid)
            path, last = self._psi.get(pid, (None, None))
            if path is None:
                path = psi_path(pid, self.proc_root)
                if path is None:
                    continue
            if path not in totals:
                totals[path] = read_psi_total_us(path)
            tot = totals[path]
            self._psi[pid] = (path, tot)
            if tot is None or last is None:
                continue
            d_ns = (tot - last) * 1000
            if d_ns >= self.floor_ns:
                rows.append((self.pod_pid(pid), pid, pod, d_ns))
        for pid in list(self._psi):
            if pid not in live:
                del self._psi[pid]
        return rows

    def tick(self, now_ns: Optional[int] = None) -> int:
        ev = self.sample(now_ns)
        if not len(ev):
            return 0
        n = int(self.push(records.to_user(ev, self.rec)))
        self.emitted += n
        self.dropped += len(ev) - n
        return n

    def start(self, interval_s: float = 0.1) -> "SchedstatSampler":
        def run():
            while not self._stop.wait(interval_s):
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
