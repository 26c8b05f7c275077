"""BPF probe loader: compiled probe objects -> loaded, attached programs sharing one set of
pinned maps (REF pkg/collector/probe_manager.go:25-185 attaches through bpf2go-generated
cilium/ebpf loaders; REF's AttachAll itself only logs, :74-86).

Every probe object (``probes/ebpf/*.bpf.o``, ``make -C probes/ebpf``) declares the same shared
maps (``mislo_probe.h``): the ring buffer, the agent-written config, the cgroup -> pod map,
the context and trace interning maps and the per-CPU scratch. They must be ONE set of maps
for the node, or the probes' ids and ring would diverge. The loader drives ``bpftool`` (the
node's libbpf: CO-RE relocation, attach-type detection) rather than re-implementing an ELF /
BTF loader:

* the first object loads with ``pinmaps <pin_dir>``, so its shared maps appear as
  ``<pin_dir>/<map>``, where ``collector/bpf.py BpfMaps`` and the agent's ring consumer open
  them;
* every later object loads with ``map name <m> pinned <pin_dir>/<m>`` for each shared map,
  reusing them;
* ``autoattach`` attaches each program by its section (kprobe/kretprobe, fentry/fexit,
  tracepoints) and pins the links under ``<pin_dir>/progs/<object>``; unloading a probe
  removes that directory, which detaches it;
* uprobe programs (``SEC("uprobe")``: no binary in the section) are only pinned by bpftool; the
  loader attaches them to every mapped instance of their library (collector/uprobes.py:
  /proc/<pid>/maps, ELF symbol offsets, perf_event_open + BPF_LINK_CREATE) and ``rescan_uprobes``
  attaches the libraries of workloads started since.

``probe_specs`` turns the objects into ``ProbeManager`` specs (one per signal; signals of one
object share a reference-counted load), so the overhead guard's shedding really detaches
programs. Needs CAP_BPF + CAP_PERFMON (root in the DaemonSet) and bpftool on the node.
"""

from __future__ import annotations

import os
import shutil
import subprocess
import threading
from typing import Callable, Dict, List, Optional, Sequence

from .probes import ProbeSpec

MISLO_SHARDS = 8  # probes/ebpf/mislo_probe.h: split rings mislo_events, mislo_events1 .. mislo_events7
# Every map mislo_probe.h pins by name, plus the per-CPU scratch: one set for the node. Later
# objects reuse them through `map name X pinned <pin_dir>/X`; a map missing here would fall back to
# libbpf's PIN_BY_NAME default root (/sys/fs/bpf), not pin_dir, and a probe could end up with a
# private shard table, staging array or split ring the agent never routes, flushes or reads.
SHARED_MAPS = (("mislo_events", "mislo_cfg", "mislo_pods", "mislo_ctxs", "mislo_traces", "mislo_scratch",
                "mislo_stages", "mislo_shards")
               + tuple(f"mislo_events{n}" for n in range(1, MISLO_SHARDS)))
# the cut's per-CPU flush of the staged batches (probes/ebpf/mislo_flush.bpf.c): loaded and pinned,
# never attached -- the agent runs it on every CPU at each window cut (collector/bpf.py BpfMaps)
FLUSH_PROBE = "mislo_flush"

# probe object -> the catalogue signals it emits (probes/ebpf/*.bpf.c)
PROBE_SIGNALS: Dict[str, Sequence[str]] = {
    "dns_latency": ("dns_latency_ms",),
    "tcp_retransmit": ("tcp_retransmits_total",),
    "runqueue_delay": ("runqueue_delay_ms",),
    "connect_latency": ("connect_latency_ms", "connect_errors_total"),
    "tls_handshake": ("tls_handshake_ms", "tls_handshake_fail_total"),
    "cpu_steal": ("cpu_steal_pct",),
    "mem_reclaim": ("mem_reclaim_latency_ms",),
    "disk_io_latency": ("disk_io_latency_ms",),
    "syscall_latency": ("syscall_latency_ms",),
    "cfs_throttle": ("cfs_throttled_ms",),
    "gpu_kfd": ("gpu_queue_delay_ms", "rccl_collective_ms"),
}


class LoaderError(RuntimeError):
    pass


class BpfProbeLoader:
    def __init__(self, obj_dir: str, pin_dir: str = "/sys/fs/bpf/mislo", bpftool: str = "bpftool",
                 run: Optional[Callable[[List[str]], None]] = None, uprobes=None, launch_uprobes: bool = False):
        self.obj_dir, self.pin_dir, self.bpftool = obj_dir, pin_dir, bpftool
        self.launch_uprobes = launch_uprobes  # per-launch HIP uprobes (collector/uprobes.py per_launch)
        self._run = run or self._subprocess
        self._lock = threading.Lock()
        self._refs: Dict[str, int] = {}
        self._uprobes = uprobes  # collector.uprobes.UprobeAttacher (created on first use)

    @property
    def uprobes(self):
        if self._uprobes is None:
            from .uprobes import UprobeAttacher

            self._uprobes = UprobeAttacher(self.pin_dir, launches=self.launch_uprobes)
        return self._uprobes

    def is_loaded(self, probe: str) -> bool:
        with self._lock:
            return self._refs.get(probe, 0) > 0

    def rescan_uprobes(self, background: bool = False) -> int:
        """Attach the loaded probes' uprobe programs to libraries mapped since the last scan
        (``background``: on the attacher's thread; returns 0 and the links appear later)."""
        from .uprobes import UPROBE_PROBES

        with self._lock:
            if not any(p in UPROBE_PROBES for p in self._refs):
                return 0
        if background:
            self.uprobes.rescan_async()
            return 0
        return self.uprobes.rescan()

    # ---- plumbing ------------------------------------------------------------------------
    @staticmethod
    def _subprocess(cmd: List[str]) -> None:
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise LoaderError(f"{' '.join(cmd)}: {r.stderr.strip() or r.stdout.strip()}")

    def obj_path(self, probe: str) -> str:
        return os.path.join(self.obj_dir, f"{probe}.bpf.o")

    def prog_dir(self, probe: str) -> str:
        return os.path.join(self.pin_dir, "progs", probe)

    def maps_pinned(self) -> bool:
        return all(os.path.exists(os.path.join(self.pin_dir, m)) for m in SHARED_MAPS)

    def available(self) -> List[str]:
        """Probe objects present in obj_dir, in PROBE_SIGNALS order."""
        return [p for p in PROBE_SIGNALS if os.path.exists(self.obj_path(p))]

    def load_cmd(self, probe: str, attach: bool = True) -> List[str]:
        cmd = [self.bpftool, "prog", "loadall", self.obj_path(probe), self.prog_dir(probe)]
        if self.maps_pinned():  # reuse the node's one set of shared maps
            for m in SHARED_MAPS:
                cmd += ["map", "name", m, "pinned", os.path.join(self.pin_dir, m)]
        else:  # first object: its shared maps become the node's
            cmd += ["pinmaps", self.pin_dir]
        return cmd + (["autoattach"] if attach else [])

    def load_flush(self) -> bool:
        """Load and pin the cut's flush program (no attachment) after the probes: without it a
        quiet CPU's partial batch stays staged until 8 slots fill, and slots more than 3 cuts old
        decode against the wrong epoch base (their 2-bit epoch tag wraps). Returns whether it is
        pinned where BpfMaps opens it."""
        if not os.path.exists(self.obj_path(FLUSH_PROBE)):
            raise LoaderError(f"no flush program {self.obj_path(FLUSH_PROBE)} (make -C probes/ebpf)")
        with self._lock:
            os.makedirs(os.path.join(self.pin_dir, "progs"), exist_ok=True)
            if os.path.exists(self.prog_dir(FLUSH_PROBE)):  # a previous agent's pin
                shutil.rmtree(self.prog_dir(FLUSH_PROBE), ignore_errors=True)
            self._run(self.load_cmd(FLUSH_PROBE, attach=False))
        return os.path.exists(os.path.join(self.prog_dir(FLUSH_PROBE), FLUSH_PROBE))

    # ---- lifecycle -------------------------------------------------------------------------
    def load(self, probe: str) -> None:
        """Load + attach ``probe`` (reference-counted: signals of one object share it)."""
        with self._lock:
            n = self._refs.get(probe, 0)
            if n == 0:
                if not os.path.exists(self.obj_path(probe)):
                    raise LoaderError(f"no probe object {self.obj_path(probe)} (make -C probes/ebpf)")
                os.makedirs(os.path.join(self.pin_dir, "progs"), exist_ok=True)
                if os.path.exists(self.prog_dir(probe)):  # a previous agent's pins
                    shutil.rmtree(self.prog_dir(probe), ignore_errors=True)
                self._run(self.load_cmd(probe))
                from .uprobes import UPROBE_PROBES

                if probe in UPROBE_PROBES:
                    self.uprobes.attach(probe)
            self._refs[probe] = n + 1

    def unload(self, probe: str) -> None:
        """Drop one reference; the last one unpins the object's programs and links (detach)."""
        with self._lock:
            n = self._refs.get(probe, 0)
            if n <= 0:
                return
            if n == 1:
                from .uprobes import UPROBE_PROBES

                if probe in UPROBE_PROBES and self._uprobes is not None:
                    self._uprobes.detach(probe)  # close the uprobe links first
                shutil.rmtree(self.prog_dir(probe), ignore_errors=True)
                del self._refs[probe]
            else:
                self._refs[probe] = n - 1

    def loaded(self) -> List[str]:
        with self._lock:
            return sorted(self._refs)


def probe_specs(loader: BpfProbeLoader, allowed: Sequence[str]) -> List[ProbeSpec]:
    """ProbeManager specs for the compiled probes serving ``allowed`` signals."""
    out = []
    for probe in loader.available():
        for sig in PROBE_SIGNALS[probe]:
            if sig in allowed:
                out.append(ProbeSpec(sig, attach=lambda p=probe: loader.load(p),
                                     detach=lambda p=probe: loader.unload(p), source="bpf"))
    return out
