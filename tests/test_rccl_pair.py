"""Two ranks of the window engine joined by one RCCL communicator (one GPU each where the box has two)
(tools/rccl_pair_probe.py), checked window by window against the CPU engine -- the oracle of every
kernel -- running the same protocol over gloo: the node-wide packet and incident features exact,
posteriors within 1e-9, the all-gathered incident results equal, both ranks' totals identical.
Skipped when RCCL refuses two ranks on one device (exit 3: a one-GPU box); the probe itself is
rehearsed on the CPU (both passes on the CPU engine) so its comparison logic runs everywhere."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _probe(engine: str, timeout: int):
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "rccl_pair_probe.py"), "--windows", "3",
                        "--engine", engine], capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert line, p.stdout[-2000:] + p.stderr[-4000:]
    return p, json.loads(line[-1])


def _assert_all_checks(p, out):
    assert p.returncode == 0, (out, p.stderr[-4000:])
    assert out["result"] == "ok", out
    assert all(out["checks"].values()), out["checks"]
    assert min(out["groups"]) > 0


@pytest.mark.timeout(300)
def test_pair_probe_rehearsal_on_the_cpu_engine():
    p, out = _probe("cpu", 280)
    _assert_all_checks(p, out)


@pytest.mark.gpu
def test_two_rank_rccl_window_engine_matches_the_cpu_oracle():
    p, out = _probe("gpu", 110)
    if p.returncode == 3:
        pytest.skip(f"RCCL refused two ranks on one device: {out.get('errors')}")
    _assert_all_checks(p, out)
