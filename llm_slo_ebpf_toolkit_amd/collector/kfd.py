"""The agent's KFD sampler (runtime/csrc/gpusampler.h): gpu_queue_delay_ms of pods whose workloads
run without the rocprofiler tool, from the amdgpu KFD driver's per-process files.

``KfdSampler`` drives the native sampler thread (occupancy readings every ``sample_s``, a decision
every ``decide_s``) and refreshes its targets -- the node's pod processes, by host pid -- from a
light Python timer, like ``procfs.NativeSampler``. When the ``gpu_kfd`` BPF object is loaded its
``hip_activity`` map (HIP runtime uprobes) tells the sampler which pods submitted GPU work, and its
kprobes report queue evictions, so the sampler's own eviction records are turned off.
"""

from __future__ import annotations

import os
import threading
from typing import Callable, Dict, Optional

import numpy as np

from . import records

KFD_PROC = "/sys/class/kfd/kfd/proc"
HIP_ACT_BYTES = 64  # probes/ebpf/mislo_record.h struct mislo_hip_act


def available(kfd_proc: str = KFD_PROC) -> bool:
    return os.path.isdir(kfd_proc)


class KfdSampler:
    def __init__(self, ring, targets: Callable[[], Dict[int, int]], node_id: int = 0, kfd_proc: str = KFD_PROC,
                 proc_root: str = "/proc", floor_pct: int = 10, sample_s: float = 0.02, decide_s: float = 0.5,
                 refresh_s: float = 10.0, hip_map: Optional[Callable[[], int]] = None, evictions: bool = True,
                 starved_hold_s: float = 1.0, stamps: int = 5):
        """``decide_s``: the contention decision's interval (its floor gates on the whole interval's
        share, so a burst of another process's kernels in one short slice does not count).
        ``stamps``: records per contended interval, the delay split evenly over them at the
        sub-intervals' middles (round 6; was one at the interval's middle): a request span joins the
        pod's records within the pod+pid tier's 100 ms of its start, so with 100 ms between records
        one is in reach wherever the start falls (config 2's second run read its first burning
        window `unknown`: no record within reach of its few request starts). ``starved_hold_s``: how
        long a pod starved of CUs stays active without a reading of its own (gpusampler.h)."""
        from ..runtime import load

        self.rt = load()
        self.targets, self.refresh_s = targets, float(refresh_s)
        self.sample_s, self.decide_s = float(sample_s), float(decide_s)
        self.native = self.rt.GpuSampler(ring, node_id=node_id, kfd_proc=kfd_proc, proc_root=proc_root,
                                         floor_pct=int(floor_pct), evictions=bool(evictions),
                                         starved_hold=max(1, int(round(starved_hold_s / max(self.decide_s, 1e-3)))),
                                         stamps=max(1, int(stamps)))
        self._hip_map = hip_map
        self._hip_fd = -1
        self._stop = threading.Event()
        self._thr: Optional[threading.Thread] = None

    # The shedding ladder's sampler rung walks the procfs signals' mask bits; gpu_queue_delay_ms is
    # shed by its GPU rung, through the ring's drop mask that the native sampler obeys like every
    # GPU producer. So this sampler reports no procfs bits and ignores the rung's mask writes.
    @property
    def mask(self) -> int:
        return 0

    @mask.setter
    def mask(self, m: int) -> None:
        pass

    @property
    def paused(self) -> bool:
        return bool(self.native.paused)

    @paused.setter
    def paused(self, p: bool) -> None:
        self.native.paused = bool(p)

    def refresh(self) -> None:
        self.native.set_target_list(sorted((int(p), int(v)) for p, v in self.targets().items()))
        if self._hip_fd < 0 and self._hip_map is not None:
            fd = int(self._hip_map())
            if fd >= 0:  # the gpu_kfd object is loaded: HIP activity from its uprobes, evictions from its kprobes
                self._hip_fd = fd
                self.native.set_hip_map(fd)

    def decide(self, now_ns: int, mono_ns: int) -> np.ndarray:
        """One decision by hand (tests): the EVENT records it produced (also pushed)."""
        return np.frombuffer(self.native.decide(int(now_ns), int(mono_ns)), dtype=records.EVENT)

    def start(self, interval_s: float = 0.0) -> "KfdSampler":
        """``interval_s`` (the procfs samplers' tick) is not this sampler's cadence: it keeps its own."""
        self.refresh()
        self.native.start(self.sample_s, self.decide_s)

        def run():
            while not self._stop.wait(self.refresh_s):
                try:
                    self.refresh()
                except Exception:  # noqa: BLE001 - keep the last target list
                    pass

        self._thr = threading.Thread(target=run, name="kfd-targets", daemon=True)
        self._thr.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        self.native.stop()
        if self._thr is not None:
            self._thr.join(5)
        if self._hip_fd >= 0:
            self.rt.close_fd(self._hip_fd)
            self._hip_fd = -1

    def stats(self) -> Dict[str, int]:
        return {f"kfd_{k}": v for k, v in dict(self.native.stats()).items()}


def hip_map_finder(loaded: Callable[[], bool]) -> Callable[[], int]:
    """The gpu_kfd object's private hip_activity map, once ``loaded()`` says the object is in."""
    def find() -> int:
        if not loaded():
            return -1
        from ..runtime import load

        return int(load().bpf_map_find("hip_activity", HIP_ACT_BYTES))
    return find
