"""rocprofiler-sdk tool library (probes/rocprof): a GPU workload with the tool loaded pushes
GPU signal records into the agent's shared-memory ring (no root, no BPF)."""

import os
import subprocess
import sys
import time

import numpy as np
import pytest

from conftest import ROOT

TOOL = os.path.join(ROOT, "llm_slo_ebpf_toolkit_amd", "probes", "rocprof", "libmislo_rocprof.so")

WORKLOAD = r"""
import torch
x = torch.randn(4096, 4096, device="cuda")
for _ in range(20):
    y = x @ x
    x = torch.tanh(y) * 0.5
keep = [torch.empty(256 << 20, dtype=torch.uint8, device="cuda") for _ in range(8)]  # 2 GiB live
torch.cuda.synchronize()
print("workload done", float(x.sum()))
"""


def test_tool_library_built():
    assert os.path.exists(TOOL), "run python -m llm_slo_ebpf_toolkit_amd.ops.build"


@pytest.mark.gpu
def test_tool_pushes_gpu_signals_into_ring():
    from llm_slo_ebpf_toolkit_amd.collector import records
    from llm_slo_ebpf_toolkit_amd.runtime import load

    rt = load()
    name = f"/mislo-test-{os.getpid()}-events"
    ring = rt.HostRing(1 << 16, 64, name)
    env = dict(os.environ, ROCP_TOOL_LIBRARIES=TOOL, MISLO_RING=name, MISLO_QUEUE_FLOOR_NS="0",
               MISLO_POD_ID="7", MISLO_NODE_ID="3", MISLO_SVC_ID="2", MISLO_ROCPROF_VERBOSE="1")
    t0 = time.time_ns()
    r = subprocess.run([sys.executable, "-c", WORKLOAD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "[mislo-rocprof] started" in r.stderr, r.stderr[-2000:]
    segs = ring.peek(1 << 16)
    view = ring.records_view()
    recs = np.concatenate([np.frombuffer(view[i * 64:(i + c) * 64].tobytes(), dtype=records.EVENT)
                           for _, i, c in segs]) if segs else np.zeros(0, dtype=records.EVENT)
    types = set(recs["signal_type"].tolist())
    assert 13 in types, (types, r.stderr[-1000:])      # gpu_queue_delay_ms from kernel dispatches
    assert 14 in types, (types, r.stderr[-1000:])      # hbm_pressure_pct from allocations
    assert (recs["pod_id"] == 7).all() and (recs["node_id"] == 3).all()
    assert (recs["flags"] & (1 << 8)).all()
    ts = recs["ts_ns"]
    assert (ts > t0 - 10 * 10**9).all() and (ts < time.time_ns() + 10 * 10**9).all()  # wall clock
    hbm = recs[recs["signal_type"] == 14]["value"].max() * 1e-3  # pct
    assert hbm > 0.5  # >= 2 GiB of 288 GiB live
