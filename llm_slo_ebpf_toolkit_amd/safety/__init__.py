"""Agent self-protection: CPU overhead guard and per-second event rate limiter.

* ``OverheadGuard`` -- REF pkg/safety/overhead_guard.go:19-158. CPU% =
  delta(utime+stime of the agent process) / delta(total ticks in /proc/stat)
  x 100 x NumCPU, i.e. percent of ONE core; the first call only primes the sampler.
  NEW: also reports RSS (MB) and the per-thread split (so GPU-runtime helper threads
  are visible, not hidden) -- used for the measured ``collector_overhead.csv``.
* ``RateLimiter`` -- REF pkg/safety/rate_limiter.go:9-39: fixed 1-second window
  counter keyed on the wall-clock second. ``TokenBucket`` is NEW and honours the
  config ``burst_limit`` that REF parses but never uses.
"""

from __future__ import annotations

import os
import sys
import threading
import time
from collections import deque
from dataclasses import dataclass
from typing import Callable, Iterable, Optional, Protocol, Tuple


@dataclass
class CPUSample:
    process_ticks: int
    total_ticks: int


class CPUSampler(Protocol):
    def sample(self) -> CPUSample: ...


def read_process_ticks(pid: int, proc_root: str = "/proc") -> int:
    with open(f"{proc_root}/{pid}/stat", "r") as fh:
        line = fh.read()
    # comm may contain spaces: split after the closing ')'
    rest = line[line.rfind(")") + 2:].split()
    # fields after comm start at index 2 (state); utime=14th, stime=15th overall
    if len(rest) < 13:
        raise ValueError(f"unexpected stat field count in {proc_root}/{pid}/stat")
    return int(rest[11]) + int(rest[12])


def read_total_ticks(proc_root: str = "/proc") -> int:
    with open(f"{proc_root}/stat", "r") as fh:
        first = fh.readline()
    fields = first.split()
    if len(fields) < 5 or fields[0] != "cpu":
        raise ValueError("unexpected cpu header in /proc/stat")
    return sum(int(f) for f in fields[1:])


def read_rss_mb(pid: int, proc_root: str = "/proc") -> float:
    try:
        with open(f"{proc_root}/{pid}/statm", "r") as fh:
            pages = int(fh.read().split()[1])
        return pages * os.sysconf("SC_PAGE_SIZE") / (1024 * 1024)
    except (OSError, ValueError, IndexError):
        return 0.0


class ProcCPUSampler:
    def __init__(self, pid: int = 0, proc_root: str = "/proc"):
        self.pid = pid if pid > 0 else os.getpid()
        self.proc_root = proc_root

    def sample(self) -> CPUSample:
        if not sys.platform.startswith("linux"):
            raise OSError("cpu sampler requires linux")
        return CPUSample(read_process_ticks(self.pid, self.proc_root), read_total_ticks(self.proc_root))


class TreeCPUSampler:
    """The agent's process tree: the controller plus its window workers (agent --gpus N). Ticks
    of processes that have exited drop out (their last reading is kept, so the sum never goes
    backwards)."""

    def __init__(self, pids: Callable[[], Iterable[int]], proc_root: str = "/proc"):
        self.pids, self.proc_root = pids, proc_root
        self._last: dict = {}

    def sample(self) -> CPUSample:
        if not sys.platform.startswith("linux"):
            raise OSError("cpu sampler requires linux")
        for pid in set(int(p) for p in self.pids()):
            try:
                self._last[pid] = read_process_ticks(pid, self.proc_root)
            except (OSError, ValueError):
                continue
        return CPUSample(sum(self._last.values()), read_total_ticks(self.proc_root))


class OverheadGuard:
    """REF's formula; with ``horizon_s`` > 0 the percentage is taken over the samples of the
    last ``horizon_s`` seconds instead of since the previous call: at 1 s evaluations 10 ms
    clock ticks quantise a sub-1 % agent to 0 or >= 1 % (a gauge reading 0.0 while the agent
    works, and shedding decisions on noise); over 30 s the resolution is 0.03 %."""

    def __init__(self, max_pct: float, sampler: Optional[CPUSampler] = None, ncpu: Optional[int] = None,
                 horizon_s: float = 0.0):
        self.max_pct = max_pct
        self.source = sampler if sampler is not None else ProcCPUSampler()
        self.ncpu = ncpu if ncpu is not None else (os.cpu_count() or 1)
        self.horizon_s = float(horizon_s)
        self._prev: Optional[CPUSample] = None
        self._hist: deque = deque()

    def evaluate(self) -> Tuple[float, bool]:
        """Returns (pct, exceeded). Raises on sampler error (REF returns err)."""
        s = self.source.sample()
        if self._prev is None:
            self._prev = s
            self._hist.append((time.monotonic(), s))
            return 0.0, False
        prev, self._prev = self._prev, s
        if self.horizon_s > 0:
            now = time.monotonic()
            self._hist.append((now, s))
            while len(self._hist) > 2 and now - self._hist[1][0] >= self.horizon_s:
                self._hist.popleft()
            prev = self._hist[0][1]
        if s.total_ticks <= prev.total_ticks:
            return 0.0, False
        d_proc = s.process_ticks - prev.process_ticks
        d_total = s.total_ticks - prev.total_ticks
        if d_total == 0:
            return 0.0, False
        pct = max((d_proc / d_total) * 100.0 * self.ncpu, 0.0)
        return pct, pct > self.max_pct


class CPUMeter:
    """Precise interval meter with the same semantics (percent of one core), using
    ``time.process_time`` (ns resolution) instead of 10 ms ticks -- for benchmarks."""

    def __init__(self):
        self._t0 = self._c0 = 0.0

    def start(self) -> None:
        self._c0 = time.process_time()
        self._t0 = time.perf_counter()

    def stop(self) -> Tuple[float, float, float]:
        cpu = time.process_time() - self._c0
        wall = time.perf_counter() - self._t0
        return (100.0 * cpu / wall if wall > 0 else 0.0), cpu, wall


class RateLimiter:
    def __init__(self, limit: int):
        self.limit = max(int(limit), 1)
        self._window = None
        self._count = 0
        self._lock = threading.Lock()

    def allow(self, now_ns: Optional[int] = None) -> bool:
        sec = (time.time_ns() if now_ns is None else now_ns) // 1_000_000_000
        with self._lock:
            if self._window != sec:
                self._window = sec
                self._count = 0
            if self._count >= self.limit:
                return False
            self._count += 1
            return True


class TokenBucket:
    """rate tokens/s refill, capacity = burst (config sampling.burst_limit)."""

    def __init__(self, rate: float, burst: int):
        self.rate = float(max(rate, 1e-9))
        self.capacity = float(max(burst, 1))
        self._tokens = self.capacity
        self._last = None
        self._lock = threading.Lock()

    def allow(self, n: int = 1, now_ns: Optional[int] = None) -> bool:
        now = (time.monotonic_ns() if now_ns is None else now_ns) / 1e9
        with self._lock:
            if self._last is not None:
                self._tokens = min(self.capacity, self._tokens + (now - self._last) * self.rate)
            self._last = now
            if self._tokens >= n:
                self._tokens -= n
                return True
            return False


class ShedLadder:
    """What the agent gives up, one step per over-budget evaluation, cheapest loss first (REF sheds
    one signal per over-budget tick in cost order, cmd/agent/main.go:587-600 with
    pkg/safety/overhead_guard.go:77-107 and pkg/signals/constants.go:46-59; REF's only lever is
    detaching a probe). The window engine's sources have cheaper levers, so the ladder is:

    1. **floors** -- every kernel probe's emit floor (``mislo_cfg`` [2 + type], read per record by
       the probes and the ring producers) rises to the signal's evidence threshold: the records
       the attribution never reads as elevated stop leaving the kernel, the elevated ones still
       arrive. One step for all probe signals.
    2. **sampler** -- the procfs sampler stops one signal per step (shed order), then pauses.
    3. **GPU producers** -- the user ring's drop mask stops one GPU signal per step (shed order);
       the rocprofiler tool inside the workloads reads it per record.
    4. **probes** -- REF's step: detach the next kernel probe (or, without loaded probes, disable
       the next signal of the synthetic generator).

    ``step()`` returns a label of what it shed, or None once nothing is left."""

    def __init__(self, order, maps=None, sampler=None, user_ring=None, probe_manager=None, generator=None):
        from ..signals import catalog

        self.order = [s for s in order if s in catalog.BY_NAME]
        self.maps, self.sampler, self.user_ring = maps, sampler, user_ring
        self.probe_manager, self.generator = probe_manager, generator
        self.floors_raised = False
        self.shed: list = []
        self._catalog = catalog

    def _floors(self) -> Optional[str]:
        if self.floors_raised or self.maps is None:
            return None
        raised = []
        for name in self.order:
            spec = self._catalog.BY_NAME[name]
            if spec.gpu or not 0 < spec.kernel_type < 120:
                continue
            raw = int(round(spec.elevated / spec.decode_scale))
            if raw > int(self.maps.cfg_get(2 + spec.kernel_type)):
                self.maps.set_floor(spec.kernel_type, raw)
                raised.append(name)
        self.floors_raised = True
        return f"floors:{','.join(raised)}" if raised else None

    def _sampler(self) -> Optional[str]:
        s = self.sampler
        if s is None or s.paused:
            return None
        from ..collector.procfs import SIGNAL_TYPES

        for name in self.order:
            t = SIGNAL_TYPES.get(name)
            if t is not None and s.mask >> t & 1:
                s.mask = s.mask & ~(1 << t)
                if s.mask == 0:
                    s.paused = True
                return f"sampler:{name}"
        s.paused = True
        return "sampler:paused"

    def _gpu(self) -> Optional[str]:
        # every worker's user ring (split rings): each GPU producer obeys the ring it writes to
        rings = self.user_ring if isinstance(self.user_ring, (list, tuple)) else [self.user_ring]
        rings = [r for r in rings if r is not None]
        if not rings:
            return None
        for name in self.order:
            spec = self._catalog.BY_NAME[name]
            if spec.gpu and not int(rings[0].drop_mask) >> spec.kernel_type & 1:
                for r in rings:
                    r.drop_mask = int(r.drop_mask) | (1 << spec.kernel_type)
                return f"gpu:{name}"
        return None

    def _probes(self) -> Optional[str]:
        pm = self.probe_manager
        sig = pm.shed_next() if pm is not None else None
        if sig:
            if self.generator is not None:
                self.generator.disable(sig)
            return f"probe:{sig}"
        if self.generator is not None:
            sig = self.generator.disable_highest_cost()
            if sig:
                return f"signal:{sig}"
        return None

    def disabled(self) -> set:
        """Signals no source emits any more (floors only thin a signal out)."""
        out = set()
        for what in self.shed:
            kind, _, name = what.partition(":")
            if kind in ("sampler", "gpu", "probe", "signal") and name in self._catalog.BY_NAME:
                out.add(name)
        if self.sampler is not None and self.sampler.paused:
            from ..collector.procfs import SIGNAL_TYPES

            out.update(SIGNAL_TYPES)
        return out

    def step(self) -> Optional[str]:
        for stage in (self._floors, self._sampler, self._gpu, self._probes):
            what = stage()
            if what:
                self.shed.append(what)
                return what
        return None
