"""BPF probe loader (collector/loader.py): the bpftool commands that load, attach and share
one set of pinned maps, reference-counted unloads, and overhead shedding that really
detaches (ProbeManager). bpftool is faked: no BPF in the container."""

import os

from llm_slo_ebpf_toolkit_amd.collector.loader import SHARED_MAPS, BpfProbeLoader, probe_specs
from llm_slo_ebpf_toolkit_amd.collector.probes import ProbeManager
from llm_slo_ebpf_toolkit_amd.signals import catalog


class FakeBpftool:
    """Records commands; creates what bpftool would pin."""

    def __init__(self):
        self.cmds = []

    def __call__(self, cmd):
        self.cmds.append(cmd)
        assert cmd[1:3] == ["prog", "loadall"]
        assert cmd[-1] == "autoattach" or cmd[3].endswith("mislo_flush.bpf.o")
        os.makedirs(cmd[4], exist_ok=True)
        open(os.path.join(cmd[4], "link0" if cmd[-1] == "autoattach" else os.path.basename(cmd[4])), "w").close()
        if "pinmaps" in cmd:
            d = cmd[cmd.index("pinmaps") + 1]
            for m in SHARED_MAPS:
                open(os.path.join(d, m), "w").close()


def _objs(tmp_path, names):
    d = tmp_path / "objs"
    d.mkdir()
    for n in names:
        (d / f"{n}.bpf.o").write_bytes(b"\x7fELF")
    return str(d)


def test_first_probe_pins_shared_maps_later_ones_reuse_them(tmp_path):
    fake = FakeBpftool()
    pin = str(tmp_path / "bpf")
    os.makedirs(pin)
    ld = BpfProbeLoader(_objs(tmp_path, ["dns_latency", "runqueue_delay"]), pin, run=fake)
    ld.load("dns_latency")
    ld.load("runqueue_delay")
    first, second = fake.cmds
    assert first[3].endswith("dns_latency.bpf.o") and first[first.index("pinmaps") + 1] == pin
    assert "pinmaps" not in second
    reused = [second[i + 2] for i, a in enumerate(second) if a == "map"]
    assert reused == list(SHARED_MAPS)
    for m in SHARED_MAPS:
        assert os.path.join(pin, m) in second
    assert ld.loaded() == ["dns_latency", "runqueue_delay"]


def test_unload_is_reference_counted_and_detaches(tmp_path):
    fake = FakeBpftool()
    pin = str(tmp_path / "bpf")
    os.makedirs(pin)
    ld = BpfProbeLoader(_objs(tmp_path, ["connect_latency"]), pin, run=fake)
    specs = probe_specs(ld, catalog.SIGNAL_NAMES)
    assert sorted(s.signal for s in specs) == ["connect_errors_total", "connect_latency_ms"]
    pm = ProbeManager(catalog.MODE_GPU, catalog.SIGNAL_NAMES)
    for s in specs:
        pm.register(s)
    assert sorted(pm.attach_all()) == ["connect_errors_total", "connect_latency_ms"]
    assert len(fake.cmds) == 1  # one object, loaded once
    prog = ld.prog_dir("connect_latency")
    assert pm.disable_probe("connect_errors_total") and os.path.isdir(prog)  # still referenced
    assert pm.disable_probe("connect_latency_ms") and not os.path.exists(prog)  # last ref: detached
    assert ld.loaded() == []


def test_overhead_shedding_detaches_in_disable_order(tmp_path):
    fake = FakeBpftool()
    pin = str(tmp_path / "bpf")
    os.makedirs(pin)
    names = ["dns_latency", "tcp_retransmit", "syscall_latency"]
    ld = BpfProbeLoader(_objs(tmp_path, names), pin, run=fake)
    pm = ProbeManager(catalog.MODE_CORE_FULL, catalog.CORE_SIGNALS)
    for s in probe_specs(ld, catalog.CORE_SIGNALS):
        pm.register(s)
    pm.attach_all()
    order = [s for s in catalog.DISABLE_ORDER if s in ("dns_latency_ms", "tcp_retransmits_total", "syscall_latency_ms")]
    shed = pm.shed_next()
    assert shed == order[0]
    gone = [p for p in names if not os.path.exists(ld.prog_dir(p))]
    assert len(gone) == 1 and shed in __import__("llm_slo_ebpf_toolkit_amd.collector.loader",
                                                 fromlist=["PROBE_SIGNALS"]).PROBE_SIGNALS[gone[0]]
    pm.detach_all()
    assert ld.loaded() == []


def test_missing_object_is_an_error(tmp_path):
    import pytest

    from llm_slo_ebpf_toolkit_amd.collector.loader import LoaderError

    ld = BpfProbeLoader(str(tmp_path), str(tmp_path / "bpf"), run=FakeBpftool())
    with pytest.raises(LoaderError):
        ld.load("dns_latency")
    assert ld.available() == []


def test_every_pinned_map_of_the_probe_header_is_shared():
    """maps pinned by name in mislo_probe.h but missing from SHARED_MAPS fall back to
    libbpf's default pin root, not pin_dir, and later objects get private copies."""
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "llm_slo_ebpf_toolkit_amd/probes/ebpf/mislo_probe.h")) as fh:
        text = fh.read()
    shards = int(re.search(r"#define MISLO_SHARDS (\d+)", text).group(1))
    pinned = set()
    for m in re.finditer(r"struct \{(.*?)\}\s*(\w+)\s*SEC\(\"\.maps\"\)", text, re.S):
        if "LIBBPF_PIN_BY_NAME" in m.group(1):
            pinned.add(m.group(2))
    if "MISLO_SHARD_RING" in text:
        pinned |= {f"mislo_events{n}" for n in range(1, shards)}
    assert pinned and pinned <= set(SHARED_MAPS), sorted(pinned - set(SHARED_MAPS))


def test_the_flush_program_is_loaded_pinned_and_never_attached(tmp_path):
    from llm_slo_ebpf_toolkit_amd.collector.loader import FLUSH_PROBE

    fake = FakeBpftool()
    pin = str(tmp_path / "bpf")
    os.makedirs(pin)
    ld = BpfProbeLoader(_objs(tmp_path, ["dns_latency", FLUSH_PROBE]), pin, run=fake)
    ld.load("dns_latency")
    assert ld.load_flush()
    cmd = fake.cmds[-1]
    assert cmd[3].endswith("mislo_flush.bpf.o") and "autoattach" not in cmd
    assert [cmd[i + 2] for i, a in enumerate(cmd) if a == "map"] == list(SHARED_MAPS)  # the node's maps
    assert os.path.exists(os.path.join(pin, "progs", FLUSH_PROBE, FLUSH_PROBE))  # where BpfMaps opens it
    assert FLUSH_PROBE not in ld.available()  # not a signal probe: shedding never detaches it
