"""`faultinject`: synthetic RawSample JSONL for collector input (REF cmd/faultinject/main.go:22-68).

Additive: ``--emit-ring PREFIX`` injects a fault at the record level into a running agent's
(emulated) BPF ring buffer instead -- the records a probe would have written for it, through the
probes' own record path (ProbeSim: definitions, trace ids, the epochs the agent publishes):

    faultinject --emit-ring /mislo-agent --signal tcp_retransmits_total --pod-uid UID \\
        --agent http://127.0.0.1:2112 --conn 51234:6333:127.0.0.1,51236:6333:127.0.0.1 --rate 40 --duration 30

The pod id is the agent's own for that pod uid (``/debug/pods``), so the records join the pod's
spans on the connection (pod + connection tier). A ``tcp_retransmits_total`` record carries the
connection's retransmits so far, as tcp_retransmit.bpf.c does.

``--fault LABEL`` injects a whole fault instead of one signal: every kernel signal of REF's
per-fault profile (pkg/signals/generator.go:244-289; the profile REF's own faultinject samples
carry), jittered like the replay (lognormal sigma 0.3, Poisson counts), one record of each per
tick -- e.g. ``network_partition``: retransmits, connect latency and errors, DNS latency, TLS
handshake failures on the victim's connections.
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
    from ..collector.otlp import _ipv4
    from ..runtime import load
    from ..signals import catalog
    from ..signals.generator import _TUPLE_SIGNALS, FAULT_OVERRIDES

    if a.fault:
        if a.fault not in FAULT_OVERRIDES:
            eprint(f"--fault {a.fault!r}: one of {sorted(FAULT_OVERRIDES)}")
            return 2
        profile = [(catalog.BY_NAME[n], v) for n, v in FAULT_OVERRIDES[a.fault].items()
                   if catalog.BY_NAME[n].kernel_type < 128]
    else:
        spec = catalog.BY_NAME.get(a.signal)
        if spec is None or spec.kernel_type >= 128:
            eprint(f"--signal {a.signal!r} is not a kernel-probe signal")
            return 2
        profile = [(spec, None)]
    pod = int(a.pod_id) if a.pod_id >= 0 else agent_pod_id(a.agent, a.pod_uid)
    conns = []
    for c in (x for x in a.conn.split(",") if x.strip()):
        sp, dp, ip = c.strip().split(":", 2)
        conns.append((int(sp), int(dp), _ipv4(ip)))
    conns = conns or [(0, 0, 0)]
    counts = [0] * len(conns)
    rt = load()
    ring = rt.Ringbuf.attach_shm(bpf.RingNames.of(a.emit_ring).ring)
    sim = rt.ProbeSim(ring, records.milli_shift_table())
    period = 1.0 / max(a.rate, 1e-3)
    n_total = int(round(a.duration * a.rate))
    rng = np.random.default_rng(a.seed)
    nxt = time.perf_counter()
    n_rec = 0
    for i in range(n_total):
        j = i % len(conns)  # connections in turn, each with its own running count
        counts[j] += 1
        ev = np.zeros(len(profile), dtype=records.EVENT)
        for r, (spec, level) in enumerate(profile):
            if level is None:  # --signal: a counter's running total, else --value
                v = counts[j] if spec.unit == "count" else a.value
            elif spec.unit == "count":
                v = max(1, int(rng.poisson(level)))
            else:
                v = level * float(np.exp(rng.normal(0.0, 0.3)))
            sport, dport, dip = conns[j] if spec.name in _TUPLE_SIGNALS or level is None else (0, 0, 0)
            ev["signal_type"][r] = spec.kernel_type
            ev["value"][r] = int(v) if spec.unit == "count" else int(round(v / spec.decode_scale))
            ev["src_port"][r], ev["dst_port"][r], ev["dst_ip"][r] = sport, dport, dip
        ev["ts_ns"] = time.time_ns()
        ev["pid"] = a.pid
        ev["tid"] = a.pid
        ev["pod_id"] = pod
        sim.submit(ev)
        n_rec += len(ev)
        nxt += period
        time.sleep(max(0.0, nxt - time.perf_counter()))
    what = f"{a.fault} fault" if a.fault else a.signal
    print(f"injected {n_rec} {what} records for pod {pod} into {a.emit_ring}", flush=True)
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
    p.flag("conn", "", "--emit-ring: sport:dport:dst-ip[,...] of the victim connection(s)")
    p.flag("rate", 20.0, "--emit-ring: records per second")
    p.flag("duration", 10.0, "--emit-ring: seconds")
    p.flag("value", 0.0, "--emit-ring: value of non-count signals (output unit, e.g. ms)")
    p.flag("fault", "", "--emit-ring: inject every kernel signal of this fault's profile (e.g. network_partition)")
    p.flag("seed", 42, "--emit-ring --fault: jitter seed")
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
