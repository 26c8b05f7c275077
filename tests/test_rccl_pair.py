"""Two ranks of the window engine joined by one RCCL communicator (one GPU each where the box has two)
(tools/rccl_pair_probe.py): the packet all-reduce gives both ranks the node-wide totals, the
incident all-gather returns every rank's own results in its slice, and the in-window trace-row
all-gather runs between the two halves of each window's chain. Skipped when RCCL refuses two
ranks on one device (exit 3: a one-GPU box)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_two_rank_rccl_window_engine():
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "rccl_pair_probe.py"), "--windows", "3"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert line, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(line[-1])
    if p.returncode == 3:
        pytest.skip(f"RCCL refused two ranks on one device: {out.get('errors')}")
    assert p.returncode == 0, (out, p.stderr[-4000:])
    assert out["result"] == "ok"
    assert out["confusion_sum"] == sum(out["groups"])
