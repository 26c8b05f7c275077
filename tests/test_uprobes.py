"""Uprobe attachment (VERDICT r2 missing #4): the TLS and RCCL uprobe programs are attached to
the libraries the node's processes map, found through /proc/<pid>/maps and addressed through
/proc/<pid>/root, at the function's file offset read from the ELF; the perf_event_open and
BPF_LINK_CREATE arguments are checked through a fake syscall layer (no privileges needed)."""

import os
import re
import shutil
import struct

import pytest

from llm_slo_ebpf_toolkit_amd.collector import uprobes as U
from llm_slo_ebpf_toolkit_amd.collector.loader import BpfProbeLoader

PROBES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "llm_slo_ebpf_toolkit_amd",
                      "probes", "ebpf")


def make_elf(path, symbols, vaddr=0x401000, foff=0x1000):
    """A minimal ELF64 shared object: one PT_LOAD (vaddr -> file offset foff) and a .dynsym
    with FUNC symbols {name: address}."""
    strtab = b"\x00"
    names = {}
    for n in symbols:
        names[n] = len(strtab)
        strtab += n.encode() + b"\x00"
    syms = b"\x00" * 24
    for n, addr in symbols.items():
        syms += struct.pack("<IBBHQQ", names[n], (1 << 4) | 2, 0, 1, addr, 16)  # GLOBAL FUNC, shndx 1
    shstr = b"\x00.dynsym\x00.dynstr\x00"
    body_off = 0x2000
    sym_off, str_off = body_off, body_off + len(syms)
    shstr_off = str_off + len(strtab)
    sh_off = (shstr_off + len(shstr) + 7) & ~7
    eh = bytearray(64)
    eh[:16] = b"\x7fELF\x02\x01\x01" + b"\x00" * 9
    struct.pack_into("<HHIQQQIHHHHHH", eh, 16, 3, 62, 1, 0, 64, sh_off, 0, 64, 56, 1, 64, 4, 3)
    ph = struct.pack("<IIQQQQQQ", 1, 5, foff, vaddr, vaddr, 0x1000, 0x1000, 0x1000)
    sh = [b"\x00" * 64,
          struct.pack("<IIQQQQIIQQ", 1, 11, 2, 0, sym_off, len(syms), 2, 1, 8, 24),
          struct.pack("<IIQQQQIIQQ", 9, 3, 2, 0, str_off, len(strtab), 0, 0, 1, 0),
          struct.pack("<IIQQQQIIQQ", 0, 3, 0, 0, shstr_off, len(shstr), 0, 0, 1, 0)]
    img = bytearray(sh_off + 64 * len(sh))
    img[:64] = eh
    img[64:64 + 56] = ph
    img[sym_off:sym_off + len(syms)] = syms
    img[str_off:str_off + len(strtab)] = strtab
    img[shstr_off:shstr_off + len(shstr)] = shstr
    for i, s in enumerate(sh):
        img[sh_off + 64 * i:sh_off + 64 * (i + 1)] = s
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as fh:
        fh.write(bytes(img))


def test_elf_symbol_offset_maps_the_address_through_its_segment(tmp_path):
    p = str(tmp_path / "libx.so")
    make_elf(p, {"SSL_do_handshake": 0x401234, "other": 0x401300})
    assert U.elf_symbol_offset(p, "SSL_do_handshake") == 0x1234
    assert U.elf_symbol_offset(p, "other") == 0x1300
    assert U.elf_symbol_offset(p, "missing") is None
    assert U.elf_symbol_offset(str(tmp_path / "nope.so"), "x") is None


def fake_proc(root, pid, libs):
    """/proc/<pid>/maps mapping ``libs`` = [(container path, dev, inode)]; the files exist under
    /proc/<pid>/root."""
    d = root / str(pid)
    os.makedirs(d / "root", exist_ok=True)
    lines = [f"55d0c0000000-55d0c0021000 r--p 00000000 fe:00 123 /usr/bin/python3\n"]
    for i, (path, dev, ino) in enumerate(libs):
        lines.append(f"7f00{i:04x}000000-7f00{i:04x}100000 r-xp 00001000 {dev} {ino}    {path}\n")
    lines.append("7ffd00000000-7ffd00021000 rw-p 00000000 00:00 0   [stack]\n")
    (d / "maps").write_text("".join(lines))


class FakeSys:
    def __init__(self):
        self.calls, self.closed, self._fd = [], [], 100

    def _next(self):
        self._fd += 1
        return self._fd

    def pmu(self):
        return (9, 0)

    def obj_get(self, path):
        self.calls.append(("obj_get", path))
        return self._next()

    def perf_uprobe_open(self, pmu_type, bit, ret, path, offset, pid=-1):
        self.calls.append(("perf", pmu_type, bit, ret, path, offset, pid))
        return self._next()

    def link_create(self, prog, perf):
        self.calls.append(("link", prog, perf))
        return self._next()

    def close(self, fd):
        self.closed.append(fd)


def test_attach_resolves_per_process_libraries_and_dedupes_by_inode(tmp_path):
    proc = tmp_path / "proc"
    # two containers mapping the same libssl file (same device + inode), one with another build
    fake_proc(proc, 101, [("/usr/lib/x86_64-linux-gnu/libssl.so.3", "08:01", 777)])
    fake_proc(proc, 202, [("/usr/lib/x86_64-linux-gnu/libssl.so.3", "08:01", 777)])
    for pid in (101, 202):
        make_elf(str(proc / str(pid) / "root/usr/lib/x86_64-linux-gnu/libssl.so.3"), {"SSL_do_handshake": 0x401a00})
    sys_ = FakeSys()
    att = U.UprobeAttacher("/sys/fs/bpf/mislo", sys_=sys_, proc_root=str(proc))
    assert att.attach("tls_handshake") == 2  # enter + exit, once for the one distinct file
    gets = [c[1] for c in sys_.calls if c[0] == "obj_get"]
    assert gets == ["/sys/fs/bpf/mislo/progs/tls_handshake/tls_enter", "/sys/fs/bpf/mislo/progs/tls_handshake/tls_exit"]
    perfs = [c for c in sys_.calls if c[0] == "perf"]
    assert [p[3] for p in perfs] == [False, True]  # entry, then the return probe
    for p in perfs:
        assert p[1:3] == (9, 0) and p[5] == 0x1a00 and p[6] == -1
        assert re.fullmatch(rf"{re.escape(str(proc))}/(101|202)/root/usr/lib/x86_64-linux-gnu/libssl\.so\.3", p[4])
    links = [c for c in sys_.calls if c[0] == "link"]
    assert [l[1] for l in links] == [101, 102]  # each program's fd onto its perf event
    assert att.links("tls_handshake") == 2 and not att.errors
    # a new workload with another libssl build: the rescan attaches just that file
    fake_proc(proc, 303, [("/lib/libssl.so.1.1", "08:02", 999)])
    make_elf(str(proc / "303/root/lib/libssl.so.1.1"), {"SSL_do_handshake": 0x402000})
    assert att.rescan() == 2 and att.rescan() == 0
    assert att.links() == 4
    att.detach("tls_handshake")
    assert att.links() == 0 and len(sys_.closed) >= 4 + 2 + 4  # perf fds, prog fds, link fds


def test_loader_attaches_uprobes_after_loading_and_detaches_on_shedding(tmp_path):
    proc = tmp_path / "proc"
    fake_proc(proc, 7, [("/opt/rocm/lib/librccl.so.1", "08:01", 4242)])
    make_elf(str(proc / "7/root/opt/rocm/lib/librccl.so.1"),
             {"ncclAllReduce": 0x401100, "ncclAllGather": 0x401200, "ncclReduceScatter": 0x401300})
    objs = tmp_path / "objs"
    objs.mkdir()
    (objs / "gpu_kfd.bpf.o").write_bytes(b"\x7fELF")
    ran = []
    sys_ = FakeSys()
    loader = BpfProbeLoader(str(objs), str(tmp_path / "pins"), run=ran.append,
                            uprobes=U.UprobeAttacher(str(tmp_path / "pins"), sys_=sys_, proc_root=str(proc)))
    loader.load("gpu_kfd")
    assert ran and ran[0][-1] == "autoattach"
    assert loader.uprobes.links("gpu_kfd") == 6  # 3 collectives x entry / return
    offs = sorted({c[5] for c in sys_.calls if c[0] == "perf"})
    assert offs == [0x1100, 0x1200, 0x1300]
    loader.unload("gpu_kfd")
    assert loader.uprobes.links() == 0


def test_uprobe_sections_name_no_binary():
    """bpftool autoattach can only pin a bare uprobe section (the agent attaches it); a section
    naming a function but no binary would fail the whole object's load."""
    for name in ("tls_handshake.bpf.c", "gpu_kfd.bpf.c"):
        src = open(os.path.join(PROBES, name)).read()
        secs = re.findall(r'SEC\("(u(?:ret)?probe[^"]*)"\)', src)
        assert secs and all(s in ("uprobe", "uretprobe") for s in secs), secs
    progs = {t.program for t in U.UPROBE_TARGETS}
    for name, probe in (("tls_handshake.bpf.c", "tls_handshake"), ("gpu_kfd.bpf.c", "gpu_kfd")):
        src = open(os.path.join(PROBES, name)).read()
        for t in U.UPROBE_TARGETS:
            if t.probe == probe:
                assert re.search(rf"\b{t.program}\b", src), t.program
    assert progs


@pytest.mark.skipif(not os.path.exists("/usr/lib/x86_64-linux-gnu/libssl.so.3"), reason="no host libssl")
def test_real_libssl_offset_is_the_exported_function():
    off = U.elf_symbol_offset("/usr/lib/x86_64-linux-gnu/libssl.so.3", "SSL_do_handshake")
    assert off is not None and off > 0


def test_rocr_and_copy_uprobes_attach_to_their_libraries(tmp_path):
    """hipMemcpy / hipMemcpyAsync get entry and return probes, ROCr's
    hsa_signal_wait_scacquire / hsa_signal_wait_relaxed (libhsa-runtime64) too."""
    proc = tmp_path / "proc"
    fake_proc(proc, 7, [("/opt/rocm/lib/libamdhip64.so.7", "08:01", 5000),
                        ("/opt/rocm/lib/libhsa-runtime64.so.1", "08:01", 5001)])
    hip = {"hipLaunchKernel": 0x401100, "hipModuleLaunchKernel": 0x401200, "hipExtModuleLaunchKernel": 0x401300,
           "hipGraphLaunch": 0x401400, "hipMemcpyAsync": 0x401500, "hipMemcpy": 0x401600,
           "hipStreamSynchronize": 0x401700, "hipDeviceSynchronize": 0x401800, "hipEventSynchronize": 0x401900}
    make_elf(str(proc / "7/root/opt/rocm/lib/libamdhip64.so.7"), hip)
    make_elf(str(proc / "7/root/opt/rocm/lib/libhsa-runtime64.so.1"),
             {"hsa_signal_wait_scacquire": 0x401a00, "hsa_signal_wait_relaxed": 0x401b00})
    sys_ = FakeSys()
    att = U.UprobeAttacher("/sys/fs/bpf/mislo", sys_=sys_, proc_root=str(proc))
    n = att.attach("gpu_kfd")
    perfs = [c for c in sys_.calls if c[0] == "perf"]
    by = {(p[4].rsplit("/", 1)[1], p[5], p[3]) for p in perfs}
    # file offsets: address - 0x401000 (the PT_LOAD's vaddr) + 0x1000 (its file offset)
    for addr in (hip["hipMemcpyAsync"], hip["hipMemcpy"]):  # the copies: entry and return
        off = addr - 0x400000
        assert ("libamdhip64.so.7", off, False) in by and ("libamdhip64.so.7", off, True) in by
    for addr in (0x401a00, 0x401b00):  # ROCr signal waits: entry and return
        off = addr - 0x400000
        assert ("libhsa-runtime64.so.1", off, False) in by and ("libhsa-runtime64.so.1", off, True) in by
    gets = {c[1].rsplit("/", 1)[1] for c in sys_.calls if c[0] == "obj_get"}
    assert {"hip_copy", "hip_copy_exit", "hsa_wait_enter", "hsa_wait_exit"} <= gets
    assert n == len(perfs) and not att.errors
    # the per-launch targets are opt-in (an LLM decode loop launches ~39,000 kernels/s)
    launch_offs = {a - 0x400000 for a in (hip["hipLaunchKernel"], hip["hipModuleLaunchKernel"],
                                          hip["hipExtModuleLaunchKernel"], hip["hipGraphLaunch"])}
    assert "hip_launch" not in gets and not launch_offs & {p[5] for p in perfs}
    sys2 = FakeSys()
    att2 = U.UprobeAttacher("/sys/fs/bpf/mislo", sys_=sys2, proc_root=str(proc), launches=True)
    assert att2.attach("gpu_kfd") == n + 4
    assert launch_offs <= {c[5] for c in sys2.calls if c[0] == "perf"}


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/libhsa-runtime64.so"), reason="no ROCm")
def test_real_rocm_wait_and_copy_symbols_resolve():
    import glob

    hsa = sorted(glob.glob("/opt/rocm/lib/libhsa-runtime64.so.*"))[-1]
    hip = sorted(glob.glob("/opt/rocm/lib/libamdhip64.so.*"))[-1]
    offs = U.elf_symbol_offsets(hsa, ["hsa_signal_wait_scacquire", "hsa_signal_wait_relaxed"])
    assert all(v > 0 for v in offs.values()) and len(offs) == 2
    offs = U.elf_symbol_offsets(hip, ["hipMemcpy", "hipMemcpyAsync"])
    assert all(v > 0 for v in offs.values()) and len(offs) == 2
