"""Uprobe attachment to the binaries the node's workloads actually map.

REF's TLS probe leaves the libssl path to its loader (/root/reference/ebpf/c/tls_handshake.bpf.c
:12-14), and no REF binary ever attaches it. A libbpf ``SEC("uprobe/<func>")`` names no binary,
so no loader can auto-attach it either. NEW's uprobe programs are declared ``SEC("uprobe")`` /
``SEC("uretprobe")``: ``bpftool prog loadall ... autoattach`` attaches the kprobes and
tracepoints of an object and merely pins its uprobe programs, and the agent attaches those
itself:

1. **resolve** -- every process's ``/proc/<pid>/maps`` names the shared objects it mapped; a
   library matching the target (``libssl.so*``, ``librccl.so*``) is addressed through
   ``/proc/<pid>/root/<path>`` (the container's mount namespace, seen from the host-PID agent),
   de-duplicated by (device, inode): one attachment per distinct file, however many processes
   and containers map it;
2. **locate** -- the function's file offset from the ELF itself (the memory-mapped file's .dynsym
   value mapped through the PT_LOAD segment that holds it), every target symbol of the library in
   one pass, cached per (device, inode);
3. **attach** -- ``perf_event_open`` on the uprobe PMU (type and retprobe bit read from
   /sys/bus/event_source/devices/uprobe) with the path and offset, then ``BPF_LINK_CREATE`` of
   the pinned program onto that perf event (runtime/csrc/bpfsys.cpp); closing the link detaches.

``UprobeAttacher.rescan_async()`` (the agent calls it with its pod rescans) attaches newly started
workloads' libraries on a background thread, off the window loop. The syscalls go through an injectable object so the argument flow is
unit-tested without privileges.
"""

from __future__ import annotations

import mmap
import os
import re
import struct
import threading
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Tuple


@dataclass(frozen=True)
class UprobeTarget:
    probe: str        # probe object (probes/ebpf/<probe>.bpf.o)
    program: str      # program name in it (pinned as progs/<probe>/<program>)
    library: str      # regex on the mapped file's basename
    symbol: str
    retprobe: bool
    # fires on every kernel launch of the probed process: opt-in (UprobeAttacher(launches=True)).
    # Measured on the demo's Llama decode (tools/uprobe_rate.py, profiles/r6_uprobe/): ~39,000
    # hipLaunchKernel calls/s, where a uprobe trap of 1-3 us each would cost the launching thread
    # 4-12 % of a core; the waits and copies fire ~13 times/s
    per_launch: bool = False


UPROBE_TARGETS: Tuple[UprobeTarget, ...] = (
    UprobeTarget("tls_handshake", "tls_enter", r"^libssl\.so", "SSL_do_handshake", False),
    UprobeTarget("tls_handshake", "tls_exit", r"^libssl\.so", "SSL_do_handshake", True),
    UprobeTarget("gpu_kfd", "allreduce_enter", r"^librccl\.so", "ncclAllReduce", False),
    UprobeTarget("gpu_kfd", "allreduce_exit", r"^librccl\.so", "ncclAllReduce", True),
    UprobeTarget("gpu_kfd", "allgather_enter", r"^librccl\.so", "ncclAllGather", False),
    UprobeTarget("gpu_kfd", "allgather_exit", r"^librccl\.so", "ncclAllGather", True),
    UprobeTarget("gpu_kfd", "reducescatter_enter", r"^librccl\.so", "ncclReduceScatter", False),
    UprobeTarget("gpu_kfd", "reducescatter_exit", r"^librccl\.so", "ncclReduceScatter", True),
    # HIP runtime: a process's GPU work submissions and its host-side waits for the GPU, per tgid
    # (gpu_kfd.bpf.c hip_activity: the agent's KFD sampler weighs other processes' occupancy of a
    # pod's GPU by them, runtime/csrc/gpusampler.h)
    UprobeTarget("gpu_kfd", "hip_launch", r"^libamdhip64\.so", "hipLaunchKernel", False, per_launch=True),
    UprobeTarget("gpu_kfd", "hip_launch", r"^libamdhip64\.so", "hipModuleLaunchKernel", False, per_launch=True),
    UprobeTarget("gpu_kfd", "hip_launch", r"^libamdhip64\.so", "hipExtModuleLaunchKernel", False, per_launch=True),
    UprobeTarget("gpu_kfd", "hip_launch", r"^libamdhip64\.so", "hipGraphLaunch", False, per_launch=True),
    UprobeTarget("gpu_kfd", "hip_copy", r"^libamdhip64\.so", "hipMemcpyAsync", False),
    UprobeTarget("gpu_kfd", "hip_copy_exit", r"^libamdhip64\.so", "hipMemcpyAsync", True),
    UprobeTarget("gpu_kfd", "hip_copy", r"^libamdhip64\.so", "hipMemcpy", False),
    UprobeTarget("gpu_kfd", "hip_copy_exit", r"^libamdhip64\.so", "hipMemcpy", True),
    UprobeTarget("gpu_kfd", "hip_sync_enter", r"^libamdhip64\.so", "hipStreamSynchronize", False),
    UprobeTarget("gpu_kfd", "hip_sync_exit", r"^libamdhip64\.so", "hipStreamSynchronize", True),
    UprobeTarget("gpu_kfd", "hip_sync_enter", r"^libamdhip64\.so", "hipDeviceSynchronize", False),
    UprobeTarget("gpu_kfd", "hip_sync_exit", r"^libamdhip64\.so", "hipDeviceSynchronize", True),
    UprobeTarget("gpu_kfd", "hip_sync_enter", r"^libamdhip64\.so", "hipEventSynchronize", False),
    UprobeTarget("gpu_kfd", "hip_sync_exit", r"^libamdhip64\.so", "hipEventSynchronize", True),
    # ROCr: the waits on GPU completion signals every blocking HIP path ends in
    UprobeTarget("gpu_kfd", "hsa_wait_enter", r"^libhsa-runtime64\.so", "hsa_signal_wait_scacquire", False),
    UprobeTarget("gpu_kfd", "hsa_wait_exit", r"^libhsa-runtime64\.so", "hsa_signal_wait_scacquire", True),
    UprobeTarget("gpu_kfd", "hsa_wait_enter", r"^libhsa-runtime64\.so", "hsa_signal_wait_relaxed", False),
    UprobeTarget("gpu_kfd", "hsa_wait_exit", r"^libhsa-runtime64\.so", "hsa_signal_wait_relaxed", True),
)
UPROBE_PROBES = frozenset(t.probe for t in UPROBE_TARGETS)


# ---------------------------------------------------------------------------------------
# ELF: function name -> file offset
# ---------------------------------------------------------------------------------------

_SYM = struct.Struct("<IBBHQQ")


def elf_symbol_offsets(path: str, symbols: Iterable[str]) -> Dict[str, int]:
    """File offsets of the defined functions among ``symbols`` in a 64-bit little-endian ELF.

    The file is memory-mapped, not read (librccl / libamdhip64 are hundreds of MB), and only the
    dynamic symbol table is walked: a uprobe target is an exported API function, which .dynsym
    always holds (.symtab -- often stripped, and 10-100x larger -- only when there is no .dynsym).
    One pass resolves every wanted name."""
    want = {w.encode(): w for w in symbols}
    out: Dict[str, int] = {}
    try:
        fh = open(path, "rb")
    except OSError:
        return out
    with fh:
        try:
            mm = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
        except (OSError, ValueError):
            return out
        with mm:
            n = len(mm)
            if n < 64 or mm[:4] != b"\x7fELF" or mm[4] != 2 or mm[5] != 1:
                return out
            e_phoff, e_shoff = struct.unpack_from("<QQ", mm, 0x20)
            e_phentsize, e_phnum, e_shentsize, e_shnum = struct.unpack_from("<HHHH", mm, 0x36)
            segs = []
            for i in range(e_phnum):
                o = e_phoff + i * e_phentsize
                if o + 56 > n:
                    break
                p_type, _f, p_offset, p_vaddr, _pa, p_filesz = struct.unpack_from("<IIQQQQ", mm, o)
                if p_type == 1:  # PT_LOAD
                    segs.append((p_vaddr, p_filesz, p_offset))
            secs = []
            for i in range(e_shnum):
                o = e_shoff + i * e_shentsize
                if o + 64 > n:
                    break
                _nm, sh_type, _fl, _ad, sh_offset, sh_size, sh_link, _in, _al, sh_entsize = \
                    struct.unpack_from("<IIQQQQIIQQ", mm, o)
                secs.append((sh_type, sh_offset, sh_size, sh_link, sh_entsize))
            tables = [x for x in secs if x[0] == 11] or [x for x in secs if x[0] == 2]  # DYNSYM, else SYMTAB
            for _t, off, size, link, ent in tables:
                if ent != 24 or link >= len(secs) or off + size > n:
                    continue
                str_off, str_size = secs[link][1], secs[link][2]
                for st_name, st_info, _o, st_shndx, st_value, _sz in _SYM.iter_unpack(mm[off:off + size - size % 24]):
                    if st_value == 0 or st_shndx == 0 or (st_info & 0xF) != 2 or st_name >= str_size:
                        continue  # defined STT_FUNC only
                    a = str_off + st_name
                    name = mm[a:mm.find(b"\x00", a, str_off + str_size)]
                    hit = want.get(name) or want.get(name.split(b"@")[0])
                    if hit is None or hit in out:
                        continue
                    for vaddr, filesz, poff in segs:
                        if vaddr <= st_value < vaddr + filesz:
                            out[hit] = st_value - vaddr + poff
                            break
                    else:
                        out[hit] = st_value
                    if len(out) == len(want):
                        return out
    return out


def elf_symbol_offset(path: str, symbol: str) -> Optional[int]:
    """File offset of one defined function (``elf_symbol_offsets`` for a single name), or None."""
    return elf_symbol_offsets(path, [symbol]).get(symbol)


# ---------------------------------------------------------------------------------------
# /proc: which processes map which library
# ---------------------------------------------------------------------------------------

_MAPS = re.compile(r"^[0-9a-f]+-[0-9a-f]+ \S+ [0-9a-f]+ ([0-9a-f]+:[0-9a-f]+) (\d+)\s+(/\S.*)$")


def mapped_libraries(pattern: str, proc_root: str = "/proc", pids: Optional[Iterable[int]] = None
                     ) -> Dict[Tuple[str, int], str]:
    """(device, inode) -> a path to that file usable from here (/proc/<pid>/root/<path>) for every
    mapped file whose basename matches ``pattern``."""
    rx = re.compile(pattern)
    out: Dict[Tuple[str, int], str] = {}
    if pids is None:
        try:
            pids = [int(p) for p in os.listdir(proc_root) if p.isdigit()]
        except OSError:
            return out
    for pid in pids:
        try:
            with open(os.path.join(proc_root, str(pid), "maps")) as fh:
                lines = fh.readlines()
        except OSError:
            continue
        for ln in lines:
            m = _MAPS.match(ln.rstrip("\n"))
            if not m:
                continue
            dev, ino, path = m.group(1), int(m.group(2)), m.group(3)
            if ino == 0 or path.endswith(" (deleted)") or not rx.search(os.path.basename(path)):
                continue
            out.setdefault((dev, ino), os.path.join(proc_root, str(pid), "root", path.lstrip("/")))
    return out


# ---------------------------------------------------------------------------------------
# attach
# ---------------------------------------------------------------------------------------

class NativeSys:
    """The real syscalls (runtime/csrc/bpfsys.cpp); every call returns an fd or -errno."""

    def __init__(self, sysfs: str = "/sys/bus/event_source/devices/uprobe"):
        from ..runtime import load

        self.rt = load()
        self.sysfs = sysfs

    def pmu(self) -> Tuple[int, int]:
        with open(os.path.join(self.sysfs, "type")) as fh:
            typ = int(fh.read().strip())
        bit = 0
        try:
            with open(os.path.join(self.sysfs, "format", "retprobe")) as fh:
                bit = int(fh.read().strip().split(":")[1])
        except (OSError, IndexError, ValueError):
            pass
        return typ, bit

    def obj_get(self, path: str) -> int:
        return self.rt.bpf_obj_get(path)

    def perf_uprobe_open(self, pmu_type: int, retprobe_bit: int, retprobe: bool, path: str, offset: int,
                         pid: int = -1) -> int:
        return self.rt.perf_uprobe_open(pmu_type, retprobe_bit, retprobe, path, offset, pid)

    def link_create(self, prog_fd: int, perf_fd: int) -> int:
        return self.rt.bpf_link_create_perf(prog_fd, perf_fd)

    def close(self, fd: int) -> None:
        self.rt.close_fd(fd)


@dataclass
class _Probe:
    progs: Dict[str, int] = field(default_factory=dict)                 # program -> prog fd
    # (program, symbol, file) -> link fd (one program may serve several functions: hip_launch)
    links: Dict[Tuple[str, str, Tuple[str, int]], int] = field(default_factory=dict)


class UprobeAttacher:
    """Attaches the pinned uprobe programs of loaded probe objects to every mapped instance of
    their libraries; ``rescan()`` picks up new ones, ``detach(probe)`` closes the links."""

    def __init__(self, pin_dir: str, sys_=None, proc_root: str = "/proc", launches: bool = False):
        """``launches``: also attach the per-launch HIP targets (``UprobeTarget.per_launch``); off by
        default -- the KFD sampler decides a pod's GPU activity from its own wave occupancy, the
        starvation hold and its waits / copies without them."""
        self.pin_dir, self.proc_root = pin_dir, proc_root
        self.launches = bool(launches)
        self.sys = sys_ if sys_ is not None else NativeSys()
        self._pmu: Optional[Tuple[int, int]] = None
        self._probes: Dict[str, _Probe] = {}
        # (dev, inode) -> {symbol: offset} of every target symbol of that library, one ELF pass
        self._offsets: Dict[Tuple[str, int], Dict[str, int]] = {}
        self._lock = threading.Lock()
        self._bg: Optional[threading.Thread] = None
        self.errors: List[str] = []

    def attach(self, probe: str) -> int:
        """Open the probe's pinned uprobe programs and attach them; returns links created."""
        with self._lock:
            st = self._probes.setdefault(probe, _Probe())
            for t in self._targets():
                if t.probe == probe and t.program not in st.progs:
                    fd = self.sys.obj_get(os.path.join(self.pin_dir, "progs", probe, t.program))
                    if fd < 0:
                        self.errors.append(f"{probe}/{t.program}: pinned program not found ({fd})")
                        continue
                    st.progs[t.program] = fd
        return self.rescan(probe)

    def _targets(self) -> Tuple[UprobeTarget, ...]:
        return tuple(t for t in UPROBE_TARGETS if self.launches or not t.per_launch)

    def rescan(self, probe: Optional[str] = None) -> int:
        """Attach to libraries mapped since the last scan; returns links created."""
        with self._lock:
            if self._pmu is None:
                self._pmu = self.sys.pmu()
            pmu_type, bit = self._pmu
            made = 0
            libs_cache: Dict[str, Dict[Tuple[str, int], str]] = {}
            for name, st in self._probes.items():
                if probe is not None and name != probe:
                    continue
                for t in self._targets():
                    if t.probe != name or t.program not in st.progs:
                        continue
                    if t.library not in libs_cache:
                        libs_cache[t.library] = mapped_libraries(t.library, self.proc_root)
                    for key, path in libs_cache[t.library].items():
                        if (t.program, t.symbol, key) in st.links:
                            continue
                        offs = self._offsets.get(key)
                        if offs is None:
                            offs = self._offsets[key] = elf_symbol_offsets(
                                path, {u.symbol for u in UPROBE_TARGETS if u.library == t.library})
                        off = offs.get(t.symbol)
                        if off is None:
                            continue  # this build of the library does not export the function
                        pfd = self.sys.perf_uprobe_open(pmu_type, bit, t.retprobe, path, off, -1)
                        if pfd < 0:
                            self.errors.append(f"{t.program} -> {path}+{off:#x}: perf_event_open {pfd}")
                            continue
                        lfd = self.sys.link_create(st.progs[t.program], pfd)
                        self.sys.close(pfd)  # the link holds the perf event
                        if lfd < 0:
                            self.errors.append(f"{t.program} -> {path}+{off:#x}: link_create {lfd}")
                            continue
                        st.links[(t.program, t.symbol, key)] = lfd
                        made += 1
            return made

    def rescan_async(self) -> bool:
        """``rescan()`` on a background thread (the /proc walk and ELF reads stay off the agent's
        window loop); False while the previous one is still running."""
        if self._bg is not None and self._bg.is_alive():
            return False

        def run():
            try:
                self.rescan()
            except Exception as e:  # a vanished process or library must not end the agent
                self.errors.append(f"rescan: {type(e).__name__}: {e}")

        self._bg = threading.Thread(target=run, name="uprobe-rescan", daemon=True)
        self._bg.start()
        return True

    def wait(self, timeout: Optional[float] = None) -> None:
        if self._bg is not None:
            self._bg.join(timeout)

    def detach(self, probe: str) -> None:
        with self._lock:
            st = self._probes.pop(probe, None)
            if st is None:
                return
            for fd in list(st.links.values()) + list(st.progs.values()):
                self.sys.close(fd)

    def links(self, probe: Optional[str] = None) -> int:
        with self._lock:
            return sum(len(st.links) for n, st in self._probes.items() if probe is None or n == probe)
