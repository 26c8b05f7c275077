"""`faultinject`: synthetic RawSample JSONL for collector input (REF cmd/faultinject/main.go:22-68).

Additive: ``--emit-ring PREFIX`` injects a fault at the record level into a running agent's
(emulated) BPF ring buffer instead -- the records a probe would have written for it, through the
probes' own record path (ProbeSim: definitions, trace ids, the epochs the agent publishes):

    faultinject --emit-ring /mislo-agent --signal tcp_retransmits_total --pod-uid UID \\
        --agent http://127.0.0.1:2112 --conn 51234:6333:127.0.0.1 --rate 40 --duration 30

The pod id is the agent's own for that pod uid (``/debug/pods``), so the records join the pod's
spans on the connection (pod + connection tier). A ``tcp_retransmits_total`` record carries the
connection's retransmits so far, as tcp_retransmit.bpf.c does.
"""

from __future__ import annotations

import json
import sys
import time
import urllib.request
from typing import List, Optional

from ..collector.pipeline import SampleMeta, generate_synthetic_samples
from ..utils.timeutil import now_ns
from ._common import GoFlags, eprint, ensure_parent, is_version_request, jsonl_line, print_version


def agent_pod_id(agent_url: str, uid: str, timeout_s: float = 30.0) -> int:
    """The agent's pod id for ``uid`` (it interns pod uids as spans and cgroups reveal them)."""
    t0 = time.time()
    while True:
        try:
            pods = json.loads(urllib.request.urlopen(agent_url.rstrip("/") + "/debug/pods", timeout=5).read())
            if uid in pods:
                return int(pods[uid])
        except (OSError, ValueError):
            pass
        if time.time() - t0 > timeout_s:
            raise RuntimeError(f"agent at {agent_url} does not know pod {uid}")
        time.sleep(0.5)


def emit_ring(a) -> int:
    import numpy as np

    from ..collector import bpf, records
    from ..runtime import load
    from ..signals import catalog

    spec = catalog.BY_NAME.get(a.signal)
    if spec is None or spec.kernel_type >= 128:
        eprint(f"--signal {a.signal!r} is not a kernel-probe signal")
        return 2
    pod = int(a.pod_id) if a.pod_id >= 0 else agent_pod_id(a.agent, a.pod_uid)
    sport = dport = dip = 0
    if a.conn:
        sp, dp, ip = a.conn.split(":", 2)
        sport, dport = int(sp), int(dp)
        from ..collector.otlp import _ipv4

        dip = _ipv4(ip)
    rt = load()
    ring = rt.Ringbuf.attach_shm(bpf.RingNames.of(a.emit_ring).ring)
    sim = rt.ProbeSim(ring, records.milli_shift_table())
    period = 1.0 / max(a.rate, 1e-3)
    n_total = int(round(a.duration * a.rate))
    count = 0
    nxt = time.perf_counter()
    for i in range(n_total):
        ev = np.zeros(1, dtype=records.EVENT)
        ev["ts_ns"] = time.time_ns()
        ev["signal_type"] = spec.kernel_type
        count += 1
        raw = count if spec.unit == "count" else int(round(a.value / spec.decode_scale))
        ev["value"] = raw
        ev["pid"] = a.pid
        ev["tid"] = a.pid
        ev["pod_id"] = pod
        ev["src_port"], ev["dst_port"], ev["dst_ip"] = sport, dport, dip
        sim.submit(ev)
        nxt += period
        time.sleep(max(0.0, nxt - time.perf_counter()))
    print(f"injected {n_total} {a.signal} records for pod {pod} into {a.emit_ring}", flush=True)
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if is_version_request(argv):
        return print_version()
    p = GoFlags("faultinject", "write synthetic raw samples")
    p.flag("scenario", "mixed", "fault injection scenario")
    p.flag("count", 24, "number of raw samples to emit")
    p.flag("out", "artifacts/fault-injection/raw_samples.jsonl", "output JSONL file for collector input")
    p.flag("cluster", "local", "cluster label")
    p.flag("namespace", "default", "namespace label")
    p.flag("workload", "gateway", "workload label")
    p.flag("service", "chat", "service label")
    p.flag("node", "kind-control-plane", "node label")
    p.flag("emit-ring", "", "inject records into a running agent's emulated BPF ring (ring name prefix)")
    p.flag("signal", "tcp_retransmits_total", "--emit-ring: the kernel signal to inject")
    p.flag("pod-uid", "", "--emit-ring: the victim pod's uid (resolved through the agent's /debug/pods)")
    p.flag("pod-id", -1, "--emit-ring: the agent's pod id, if known (skips the lookup)")
    p.flag("agent", "http://127.0.0.1:2112", "--emit-ring: the agent's metrics address")
    p.flag("pid", 0, "--emit-ring: pid on the records (0: none, e.g. softirq-context retransmits)")
    p.flag("conn", "", "--emit-ring: sport:dport:dst-ip of the victim connection")
    p.flag("rate", 20.0, "--emit-ring: records per second")
    p.flag("duration", 10.0, "--emit-ring: seconds")
    p.flag("value", 0.0, "--emit-ring: value of non-count signals (output unit, e.g. ms)")
    a = p.parse_args(argv)
    if a.emit_ring:
        try:
            return emit_ring(a)
        except (RuntimeError, OSError, ValueError) as exc:
            eprint(f"fault injection failed: {exc}")
            return 1
    meta = SampleMeta(cluster=a.cluster, namespace=a.namespace, workload=a.workload, service=a.service,
                      node=a.node)
    try:
        samples = generate_synthetic_samples(a.scenario, a.count, now_ns(), meta)
    except ValueError as exc:
        eprint(f"generate fault-injection samples failed: {exc}")
        return 1
    ensure_parent(a.out)
    with open(a.out, "w", encoding="utf-8") as fh:
        for s in samples:
            fh.write(jsonl_line(s))
    print(f"wrote {len(samples)} raw samples to {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
