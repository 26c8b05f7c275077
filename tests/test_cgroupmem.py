"""utils/cgroupmem.py: a process's memory-cgroup charge read from v1 and v2 hierarchies (scripted
trees; the real reading is exercised by tools/agent_overhead.py and tools/queue_mem_probe.py)."""

import os

from llm_slo_ebpf_toolkit_amd.utils import cgroupmem


def _proc_cgroup(tmp_path, text):
    # reading() takes a pid; a scripted /proc/<pid>/cgroup is not possible, so patch open's target
    p = tmp_path / "cgroup"
    p.write_text(text)
    return str(p)


def test_v2_charge_and_stat(tmp_path, monkeypatch):
    root = tmp_path / "fs"
    d = root / "kubepods" / "pod1"
    d.mkdir(parents=True)
    (d / "memory.current").write_text("104857600\n")
    (d / "memory.stat").write_text("anon 52428800\nfile 10485760\nshmem 4194304\nkernel 1048576\nother 7\n")
    cg = _proc_cgroup(tmp_path, "0::/kubepods/pod1\n")
    real_open = open
    monkeypatch.setattr("builtins.open", lambda f, *a, **k: real_open(cg if f == "/proc/self/cgroup" else f, *a, **k))
    r = cgroupmem.reading("self", str(root))
    assert r["version"] == 2 and r["dir"] == str(d) and r["charged_bytes"] == 100 << 20
    assert r["stat"] == {"anon": 50 << 20, "file": 10 << 20, "shmem": 4 << 20, "kernel": 1 << 20}
    (d / "memory.current").write_text(str((100 << 20) + (30 << 20)))
    (d / "memory.stat").write_text("anon 83886080\nfile 10485760\nshmem 4194304\nkernel 1048576\n")
    assert cgroupmem.delta(r, cgroupmem.reading("self", str(root))) == {
        "charged_mb": 30.0, "anon_mb": 30.0, "file_mb": 0.0, "shmem_mb": 0.0, "kernel_mb": 0.0}


def test_v1_memory_controller_and_namespace_root(tmp_path, monkeypatch):
    root = tmp_path / "fs"
    m = root / "memory"  # inside a cgroup namespace the named path is absent: the root is ours
    m.mkdir(parents=True)
    (m / "memory.usage_in_bytes").write_text("2097152\n")
    (m / "memory.stat").write_text("cache 1048576\nrss 524288\nshmem 0\nmapped_file 0\ntotal_rss 9\n")
    cg = _proc_cgroup(tmp_path, "4:memory:/process_api/abc\n3:cpuset:/\n0::/\n")
    real_open = open
    monkeypatch.setattr("builtins.open", lambda f, *a, **k: real_open(cg if f == "/proc/self/cgroup" else f, *a, **k))
    r = cgroupmem.reading("self", str(root))
    assert r["version"] == 1 and r["dir"] == str(m) and r["charged_bytes"] == 2 << 20
    assert r["stat"] == {"cache": 1 << 20, "rss": 1 << 19, "shmem": 0, "mapped_file": 0}


def test_no_memory_cgroup(tmp_path, monkeypatch):
    cg = _proc_cgroup(tmp_path, "1:cpu:/\n")
    real_open = open
    monkeypatch.setattr("builtins.open", lambda f, *a, **k: real_open(cg if f == "/proc/self/cgroup" else f, *a, **k))
    assert cgroupmem.reading("self", str(tmp_path / "none")) is None
    assert cgroupmem.delta(None, None) is None
    assert os.path.exists(cg)
