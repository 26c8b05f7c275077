"""`agent`: node DaemonSet process (REF cmd/agent/main.go:269-633; flags :334-373).

REF flags are all accepted with REF defaults. Additive flags select the MI355X window
engine: ``--engine gpu|cpu --source bpf|shm|replay --gpus --pin-dir --window-ms --window-events
--device --model --model-path --min-confidence --ttft-slo-ms --slo-target``; ``--count`` bounds the
number of windows in window-engine mode.
"""

from __future__ import annotations

import faulthandler
import os
import signal
import sys
from typing import List, Optional

from ..agent.daemon import Agent, AgentOptions, run_forever
from ..collector.probes import probe_smoke_check
from ._common import GoFlags, eprint, is_version_request, print_version, split_csv


ENGINES = ("synthetic", "gpu", "cpu")
SOURCES = ("bpf", "shm", "replay")
MODELS = ("bayes", "bayes_gpu", "bayes_learned", "lda")


def parse(argv: List[str]) -> (AgentOptions, bool):
    d = AgentOptions()
    p = GoFlags("agent", "LLM SLO node agent (MI355X window engine)")
    # the additive flags are checked at parse time; REF's own flags keep REF's post-parse
    # validation (exit 1, cmd/agent/main.go)
    choices = {"engine": ENGINES, "source": SOURCES, "model": MODELS}
    for name, default, help_ in [
        ("cluster", d.cluster, "cluster name"), ("namespace", d.namespace, "namespace"),
        ("workload", d.workload, "workload"), ("service", d.service, "service"),
        ("k8s-node", d.node, "node label"), ("pod", d.pod, "pod name"), ("container", d.container, "container name"),
        ("scenario", d.scenario, "synthetic scenario name"), ("count", d.count, "sample count (0 = stream mode)"),
        ("interval-ms", d.interval_ms, "emit interval for stream mode"),
        ("event-kind", d.event_kind, "event kind: slo|probe|both"),
        ("output", d.output, "output mode: stdout|jsonl|otlp"),
        ("output-path", d.output_path, "output file when output=jsonl"),
        ("otlp-endpoint", d.otlp_endpoint, "OTLP/HTTP logs endpoint when output=otlp"),
        ("otlp-timeout-ms", d.otlp_timeout_ms, "OTLP export timeout in milliseconds"),
        ("otlp-batch", d.otlp_batch, "log records per OTLP POST"),
        ("webhook-url", d.webhook_url, "webhook endpoint URL (empty = disabled)"),
        ("webhook-secret", d.webhook_secret, "HMAC-SHA256 secret for webhook signing"),
        ("webhook-format", d.webhook_format, "webhook payload format: generic|pagerduty|opsgenie"),
        ("webhook-timeout-ms", d.webhook_timeout_ms, "webhook HTTP timeout in milliseconds"),
        ("capability-mode", d.capability_mode, "capability mode: auto|core_full|bcc_degraded|replay|gpu"),
        ("disable-signals", "", "comma-separated signal names to disable"),
        ("disable-overhead-guard", False, "disable overhead guard"),
        ("config", d.config, "toolkit config path"),
        ("enable-hello-tracer", False, "enable hello tracer metric path"),
        ("hello-target-comm", ",".join(d.hello_target_comm), "comma-separated comm names for hello tracer"),
        ("enable-real-probe-metrics", True, "enable probe-derived metrics on /metrics"),
        ("metrics-bind", d.metrics_bind, "metrics and health bind address"),
        ("probe-smoke", False, "run eBPF smoke check and exit"),
        ("engine", d.engine, "attribution engine: synthetic (REF tick loop) | gpu (MI355X window engine) | cpu "
                             "(the window engine's contract on the host: the numpy oracle; hosts without a GPU)"),
        ("source", d.source, "window engine record source: bpf (pinned probe maps) | shm (emulated rings) | replay"),
        ("gpus", d.gpus, "window workers, one per GPU (0 = every GPU visible to the agent); each owns a share of "
                         "the node's services, node-wide results over RCCL"),
        ("split-rings", True, "with --gpus N > 1: one ring set per worker, every producer routing each record to "
                              "the worker owning its service (false: every worker reads the whole stream)"),
        ("model-path", d.model_path, "trained attribution model (safetensors) written by `attributor --train`; "
                                     "overrides --model"),
        ("otlp-receiver-allow", d.otlp_receiver_allow, "comma-separated CIDRs allowed to export spans to the "
                                                       "receiver (empty = any)"),
        ("otlp-forwarders", d.otlp_forwarders, "comma-separated CIDRs of trusted span forwarders (an OTel collector "
                                               "relaying other pods' spans): exempt from the check that a span "
                                               "naming a pod comes from that pod's address"),
        ("procfs-sampler", False, "window engine: run-queue delay, CPU wait share (cpu_steal_pct), CFS throttling "
                                  "and memory stall of pod processes from /proc schedstat and their cgroups "
                                  "(unprivileged; min-capability mode)"),
        ("procfs-pods", d.procfs_pods, "pid:pod-uid,... for the procfs sampler (empty: the kubepods cgroups)"),
        ("procfs-interval-ms", d.procfs_interval_ms, "procfs sampler interval"),
        ("kfd-sampler", d.kfd_sampler, "gpu_queue_delay_ms from the KFD driver's per-process files: other processes' "
                                       "wave occupancy of a pod's GPU and its queue evictions (auto | on | off; "
                                       "auto = when /sys/class/kfd exists and pod processes are watched)"),
        ("procfs-cpu-psi", False, "procfs sampler: cpu_steal_pct is also the pod cgroup's cpu.pressure 'some' share "
                                  "(pod-private cgroups only)"),
        ("model-signals", d.model_signals, "window engine: comma-separated signals this node's sources produce; "
                                           "the model sums the others out instead of reading their absence as "
                                           "'not elevated' (empty = every signal)"),
        ("retrieval-residual-ms", d.retrieval_residual_ms, "window engine: application evidence -- an incident "
                                                           "group whose spans' retrieval time (llm.slo.retrieval.*) "
                                                           "exceeds the kernel-attributed share (dns + connect + "
                                                           "TLS) by at least this is retrieval_backend evidence "
                                                           "(<= 0 = off)"),
        ("hip-launch-uprobes", False, "bpf source: also uprobe every HIP kernel launch (hipLaunchKernel & co.) "
                                      "for the KFD sampler's activity decision; off by default -- an LLM decode "
                                      "loop launches ~39,000 kernels/s and each uprobe hit traps (1-3 us)"),
        ("pair-prior", d.pair_prior, "window engine: add 2-fault hypotheses with this prior mass to a table model "
                                     "(--model bayes | bayes_gpu; trained files carry their own)"),
        ("ring-name", d.ring_name, "shared-memory ring name prefix (user-space / span rings; emulated BPF ring)"),
        ("pin-dir", d.pin_dir, "bpffs directory the probe loader pinned the maps in (--source bpf)"),
        ("probe-objs", d.probe_objs, "--source bpf: directory of compiled probes (*.bpf.o) the agent loads and "
                                     "attaches with bpftool, pinning their shared maps in --pin-dir "
                                     "(empty: an external loader did)"),
        ("window-ms", d.window_ms, "gpu engine window length"),
        ("window-events", d.window_events, "gpu engine events per window (capacity)"),
        ("window-spans", d.window_spans, "gpu engine spans per window (capacity)"),
        ("window-groups", d.window_groups, "gpu engine incident groups per window"),
        ("device", d.device, "HIP device ordinal"),
        ("model", d.model, "attribution model: bayes (REF table) | bayes_gpu (REF table + GPU signals/domains) | bayes_learned | lda"),
        ("min-confidence", d.min_confidence, "emit incidents whose top posterior is at least this"),
        ("ttft-slo-ms", d.ttft_slo_ms, "per-incident TTFT SLO (ms) for burn rates"),
        ("slo-target", d.slo_target, "TTFT SLO objective for burn rates (0.99 = 1%% error budget)"),
        ("otlp-receiver-bind", d.otlp_receiver_bind, "OTLP/HTTP /v1/traces receiver feeding the span ring (gpu engine)"),
        ("halo-ms", d.halo_ms, "gpu engine: records this close to a window's end also join the next window (0 = off)"),
        ("state-dir", d.state_dir, "gpu engine: checkpoint directory for the learned state (resumed on start)"),
        ("checkpoint-every", d.checkpoint_every, "gpu engine: windows between checkpoints"),
        ("emit-wait-ms", d.emit_wait_ms, "gpu engine: after a cut, wait up to this long for the window's results "
                                         "and emit them at once (0 = with the next cut)"),
        ("webhook-queue", d.webhook_queue, "attributions queued for webhook delivery (more are dropped)"),
        ("emit-min-burn", d.emit_min_burn, "gpu engine: attribute an incident group only while its SLO burn rate "
                                           "(error-budget multiples) is at least this (<= 0: every scored group)"),
        ("emit-min-requests", d.emit_min_requests, "gpu engine: the emission gate's burn is over the last windows "
                                                   "(at most 3) holding this many requests"),
        ("emit-recovered-requests", d.emit_recovered_requests, "gpu engine: a window that completes at least "
                                                               "this many requests of a group, none breaching "
                                                               "its SLO in the window, is not attributed (0 = off, "
                                                               "-1 = 4 per second of window, at least 2)"),
        ("decision-log", d.decision_log, "gpu engine: JSONL of every scored incident group per window -- "
                                         "requests, breaches, burn, top posteriors, emitted or why not (\"\" = off)"),
        ("gpu-hw-queues", 1, "gpu engine: cap on HIP hardware queues (GPU_MAX_HW_QUEUES; the flag given on the "
                             "command line wins over the env, the default does not; "
                             "each MI355X queue pins ~173 MB of host memory; 1 serialises copy and compute, ample "
                             "at node event rates; 0 = runtime default)"),
    ]:
        p.flag(name, default, help_, choices=choices.get(name))
    a = p.parse_args(argv)
    o = AgentOptions(
        cluster=a.cluster, namespace=a.namespace, workload=a.workload, service=a.service, node=a.k8s_node,
        pod=a.pod, container=a.container, scenario=a.scenario, count=a.count, interval_ms=a.interval_ms,
        event_kind=a.event_kind, output=a.output, output_path=a.output_path, otlp_endpoint=a.otlp_endpoint,
        otlp_timeout_ms=a.otlp_timeout_ms, otlp_batch=a.otlp_batch, webhook_url=a.webhook_url,
        webhook_secret=a.webhook_secret, webhook_format=a.webhook_format, webhook_timeout_ms=a.webhook_timeout_ms,
        capability_mode=a.capability_mode, disable_signals=split_csv(a.disable_signals),
        disable_overhead_guard=a.disable_overhead_guard, config=a.config, enable_hello_tracer=a.enable_hello_tracer,
        hello_target_comm=split_csv(a.hello_target_comm), enable_real_probe_metrics=a.enable_real_probe_metrics,
        metrics_bind=a.metrics_bind, engine=a.engine, source=a.source, ring_name=a.ring_name, pin_dir=a.pin_dir,
        probe_objs=a.probe_objs,
        window_ms=a.window_ms, window_events=a.window_events, window_spans=a.window_spans,
        window_groups=a.window_groups, device=a.device, model=a.model, min_confidence=a.min_confidence,
        ttft_slo_ms=a.ttft_slo_ms, slo_target=a.slo_target,
        otlp_receiver_bind=a.otlp_receiver_bind, halo_ms=float(a.halo_ms), state_dir=a.state_dir,
        checkpoint_every=int(a.checkpoint_every), gpus=int(a.gpus), split_rings=bool(a.split_rings), model_path=a.model_path,
        otlp_receiver_allow=a.otlp_receiver_allow, otlp_forwarders=a.otlp_forwarders, procfs_sampler=bool(a.procfs_sampler), procfs_pods=a.procfs_pods,
        procfs_interval_ms=int(a.procfs_interval_ms), procfs_cpu_psi=bool(a.procfs_cpu_psi),
        kfd_sampler=a.kfd_sampler,
        model_signals=a.model_signals, retrieval_residual_ms=float(a.retrieval_residual_ms),
        hip_launch_uprobes=bool(a.hip_launch_uprobes),
        pair_prior=float(a.pair_prior), emit_wait_ms=int(a.emit_wait_ms), webhook_queue=int(a.webhook_queue),
        emit_min_burn=float(a.emit_min_burn), emit_min_requests=float(a.emit_min_requests),
        emit_recovered_requests=int(a.emit_recovered_requests),
        decision_log=a.decision_log,
        explicit_flags=tuple(sorted({x.lstrip("-").split("=", 1)[0] for x in (argv if argv is not None else sys.argv[1:]) if x.startswith("-")})))
    if int(a.gpu_hw_queues) > 0:  # before anything initialises the HIP runtime
        given = any(x.lstrip("-").split("=", 1)[0] == "gpu-hw-queues" for x in argv or [])
        if given:  # an operator's flag wins over a node-wide GPU_MAX_HW_QUEUES
            os.environ["GPU_MAX_HW_QUEUES"] = str(int(a.gpu_hw_queues))
        else:
            os.environ.setdefault("GPU_MAX_HW_QUEUES", str(int(a.gpu_hw_queues)))
    if os.environ.get("GPU_MAX_HW_QUEUES") == "1":
        # one hardware queue runs a copy stream's and the compute stream's commands in order
        # anyway: one HIP stream (its second stream's host state is ~16 MB), and the window's
        # host->device copies as blit kernels on that queue instead of SDMA -- the first large SDMA
        # copy maps another 173.4 MB queue save area into the process (tools/native/hip_rss_floor.hip,
        # profiles/r5_rss/); the agent copies ~20 MB/s at 1M events/s, far below either path's rate
        os.environ.setdefault("MISLO_ONE_STREAM", "1")
        os.environ.setdefault("HSA_ENABLE_SDMA", "0")
    return o, a.probe_smoke


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    try:  # operators: `kill -USR1 <pid>` dumps every thread's stack to stderr
        faulthandler.register(signal.SIGUSR1, all_threads=True)
    except (AttributeError, ValueError, OSError):  # no SIGUSR1, or stderr is not a real file
        pass
    if is_version_request(argv):
        return print_version()
    opts, smoke = parse(argv)
    if smoke:
        try:
            probe_smoke_check()
        except Exception as exc:  # noqa: BLE001
            eprint(f"probe smoke failed: {exc}")
            return 1
        print("probe smoke ok")
        return 0
    try:
        agent = Agent(opts)
    except Exception as exc:  # noqa: BLE001
        eprint(str(exc))
        return 1
    agent.start_server()
    agent.start_hello_tracer()
    if opts.engine in ("gpu", "cpu"):
        if opts.engine == "gpu":
            from ..ops import load_agent

            # the native engine must be built: fail loudly, never fall back (import only: this
            # process forks the replay producer and spawns the GPU workers; it never initialises HIP)
            load_agent(init=False)
        try:
            return run_forever(agent, lambda: agent.run_windows(max_windows=opts.count))
        except Exception as exc:  # noqa: BLE001 - a worker or source failure ends the agent (k8s restarts it)
            eprint(f"window engine failed: {exc}")
            return 1
    try:
        return run_forever(agent, agent.run_synthetic)
    except Exception as exc:  # noqa: BLE001 - REF: emit failures are fatal (exit 1)
        eprint(f"emit sample failed: {exc}")
        return 1


if __name__ == "__main__":
    sys.exit(main())
