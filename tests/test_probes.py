"""Probe sources: record layout shared with the ring / GPU decoder, and every catalogue
signal has a producer whose program names exist in its source."""

import os
import re
import shutil
import subprocess

import pytest

from llm_slo_ebpf_toolkit_amd.probes import EBPF_DIR, PROBES
from llm_slo_ebpf_toolkit_amd.signals import catalog


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs a host C compiler")
def test_bpf_record_layout_matches_event_dtype(tmp_path):
    exe = tmp_path / "layout_check"
    subprocess.run(["gcc", "-Wall", "-I", EBPF_DIR, "-o", str(exe), os.path.join(EBPF_DIR, "layout_check.c")],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    # the in-kernel fixed-point rule (mislo_milli) == records.milli_int
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.collector import records

    rows = [tuple(int(x) for x in ln.split()[1:]) for ln in out.stdout.splitlines() if ln.startswith("milli ")]
    assert len(rows) == 52
    t, v, m = (np.array(c, dtype=np.uint64) for c in zip(*rows))
    shift = records.milli_shift_table()[t.astype(np.int64)]
    np.testing.assert_array_equal(records.milli_int(v, shift), m.astype(np.uint32))


def test_record_enum_matches_catalogue():
    src = open(os.path.join(EBPF_DIR, "mislo_record.h")).read()
    enum = {int(v): k for k, v in re.findall(r"MISLO_(\w+) = (\d+)", src)}
    for s in catalog.SIGNALS:
        assert s.kernel_type in enum, s.name
    assert catalog.HELLO_TYPE in enum


def test_every_signal_has_a_producer():
    for s in catalog.SIGNALS:
        assert s.name in PROBES, s.name
    for sig, (kind, obj, progs) in PROBES.items():
        if "bpf" not in kind:
            continue
        src = open(os.path.join(EBPF_DIR, obj + ".bpf.c")).read()
        for p in progs:
            assert re.search(rf"\b{p}\b\s*[(,)]", src), (sig, obj, p)
        assert 'SEC("license")' in src
