"""Probe lifecycle: probe manager, kernel smoke check, BCC-degraded fallback, hello tracer.

* ``ProbeManager`` -- REF pkg/collector/probe_manager.go:15-185: registry of probes
  allowed for a capability mode, disable-by-name, overhead-driven shedding in the
  configured disable order. REF's ``AttachAll`` only logs (:74-86); here a probe is a
  ``ProbeSpec`` with real ``attach``/``detach`` callables (a BPF loader, a
  rocprofiler-sdk tool session, a /proc poller or a replay source), so shedding
  actually stops the source.
* ``probe_smoke_check`` -- REF kernel.go:18-39: Linux + root + create a 1-entry BPF
  hash map. Implemented with the raw bpf(2) syscall via ctypes (no libbpf needed).
* ``BCCFallback`` -- REF bcc_fallback.go:14-74 capability flags (dns + tcp only).
* ``HelloTracer`` -- REF hello_tracer.go:42-86 (timer-driven per-comm counter).
"""

from __future__ import annotations

import ctypes
import logging
import os
import platform
import struct
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

from ..signals import catalog

log = logging.getLogger(__name__)


@dataclass
class ProbeSpec:
    signal: str
    attach: Optional[Callable[[], None]] = None
    detach: Optional[Callable[[], None]] = None
    attached: bool = False
    source: str = "bpf"  # bpf | rocprofiler | procfs | replay


class ProbeManager:
    def __init__(self, mode: str, allowed: Sequence[str], disable_order: Sequence[str] = catalog.DISABLE_ORDER,
                 guard=None, limiter=None):
        self._lock = threading.Lock()
        self.mode = mode
        self._allowed = set(allowed)
        self.disable_order = list(disable_order)
        self.guard = guard
        self.limiter = limiter
        self._probes: Dict[str, ProbeSpec] = {}

    def register(self, spec: ProbeSpec) -> None:
        with self._lock:
            if spec.signal not in self._allowed:
                raise ValueError(f'signal "{spec.signal}" not supported in mode {self.mode}')
            self._probes[spec.signal] = spec

    def attach_all(self) -> List[str]:
        done = []
        with self._lock:
            for sig, spec in self._probes.items():
                if spec.attached:
                    continue
                if spec.attach is not None:
                    spec.attach()
                spec.attached = True
                done.append(sig)
                log.info("probe %s: attached (%s)", sig, spec.source)
        return done

    def _close(self, sig: str, spec: ProbeSpec) -> None:
        if spec.detach is not None and spec.attached:
            try:
                spec.detach()
            except Exception as exc:  # never fatal, like REF's link close errors
                log.warning("probe %s: detach error: %s", sig, exc)
        spec.attached = False
        log.info("probe %s: detached", sig)

    def detach_all(self) -> None:
        with self._lock:
            for sig, spec in self._probes.items():
                self._close(sig, spec)
            self._probes = {}

    def disable_probe(self, signal: str) -> bool:
        with self._lock:
            spec = self._probes.pop(signal, None)
            if spec is None:
                return False
            self._close(signal, spec)
            return True

    def enabled_signals(self) -> List[str]:
        with self._lock:
            return list(self._probes)

    def check_overhead(self) -> Optional[str]:
        """Evaluate the guard; when over budget shed the next probe in disable order."""
        if self.guard is None:
            return None
        try:
            pct, exceeded = self.guard.evaluate()
        except Exception as exc:
            log.warning("overhead check error: %s", exc)
            return None
        if not exceeded:
            return None
        log.warning("overhead %.2f%% exceeds budget, disabling highest-cost probe", pct)
        return self.shed_next()

    def shed_next(self) -> Optional[str]:
        """Detach the next enabled probe in disable order (REF disableHighestCostProbe)."""
        with self._lock:
            for sig in self.disable_order:
                spec = self._probes.pop(sig, None)
                if spec is not None:
                    self._close(sig, spec)
                    return sig
        return None


# --- bpf(2) smoke check -----------------------------------------------------------------

_BPF_MAP_CREATE = 0
_BPF_MAP_TYPE_HASH = 1
_SYS_BPF = {"x86_64": 321, "aarch64": 280}


def probe_smoke_check() -> None:
    """Raise OSError unless a 1-entry BPF hash map can be created (REF kernel.go:18-39)."""
    if not sys.platform.startswith("linux"):
        raise OSError("probe smoke requires linux host")
    if os.geteuid() != 0:
        raise OSError("probe smoke requires privileged execution")
    nr = _SYS_BPF.get(platform.machine())
    if nr is None:
        raise OSError(f"unsupported architecture {platform.machine()}")
    libc = ctypes.CDLL(None, use_errno=True)
    attr = ctypes.create_string_buffer(struct.pack("IIIII", _BPF_MAP_TYPE_HASH, 4, 4, 1, 0) + b"\0" * 108)
    fd = libc.syscall(nr, _BPF_MAP_CREATE, attr, 120)
    if fd < 0:
        err = ctypes.get_errno()
        raise OSError(err, f"create smoke map: {os.strerror(err)}")
    os.close(fd)


class BCCFallback:
    def __init__(self):
        self.active = False

    @staticmethod
    def supported_signals() -> List[str]:
        return list(catalog.BCC_SIGNALS)

    def start(self) -> None:
        if self.active:
            raise RuntimeError("bcc fallback already active")
        log.info("bcc fallback: starting degraded mode with %d signals", len(catalog.BCC_SIGNALS))
        self.active = True

    def stop(self) -> None:
        if self.active:
            log.info("bcc fallback: stopping degraded mode")
        self.active = False

    def capability_flags(self) -> Dict[str, object]:
        return {"mode": catalog.MODE_BCC_DEGRADED, "supported_signals": self.supported_signals(),
                "degraded": True, "note": "BCC fallback: DNS and TCP retransmits only; CO-RE unavailable"}


@dataclass
class HelloEvent:
    timestamp: int
    comm: str
    count: int


def sanitize_targets(targets: Sequence[str]) -> List[str]:
    seen = set()
    out = []
    for t in targets:
        v = t.strip()
        if v and v not in seen:
            seen.add(v)
            out.append(v)
    return out


class HelloTracer:
    def __init__(self, targets: Sequence[str], interval_s: float = 2.0):
        self.targets = sanitize_targets(targets)
        self.interval_s = interval_s if interval_s > 0 else 2.0

    def start(self, stop: threading.Event, emit: Callable[[HelloEvent], None]) -> None:
        if emit is None or not self.targets:
            return
        while True:
            ts = time.time_ns()
            for comm in self.targets:
                emit(HelloEvent(ts, comm, 1))
            if stop.wait(self.interval_s):
                return
