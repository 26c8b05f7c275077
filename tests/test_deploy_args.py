"""The shipped deployments start: the Helm chart's and the kustomize
DaemonSet's agent arguments, rendered with their own values / ConfigMap, parse with the agent's
CLI into options the window engine accepts; the learned model they point at is the one
`attributor --train` produces; the helm test pod is well formed."""

import os
import re

import numpy as np
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIPPED_MODEL = "config/models/mislo-learned.safetensors"


def _get(values, dotted):
    v = values
    for part in dotted.split("."):
        v = v[part]
    return v


def render_chart_args():
    """The chart's container args with `{{ .Values.* }}` substituted from values.yaml (the chart
    uses no other construct in its args; `range .Values.agent.extraArgs` expands the list)."""
    with open(os.path.join(ROOT, "charts/llm-slo-agent/values.yaml")) as fh:
        values = yaml.safe_load(fh)
    with open(os.path.join(ROOT, "charts/llm-slo-agent/templates/daemonset.yaml")) as fh:
        text = fh.read()
    block = text[text.index("          args:\n"):text.index("          env:")]
    args = []
    in_range = False
    for ln in block.splitlines()[1:]:
        s = ln.strip()
        if s.startswith("{{- range .Values.agent.extraArgs"):
            in_range = True
            args += [str(x) for x in values["agent"]["extraArgs"]]
            continue
        if s.startswith("{{- end"):
            in_range = False
            continue
        if in_range or not s.startswith("- "):
            continue
        arg = re.sub(r"\{\{\s*\.Values\.([\w.]+)\s*\}\}", lambda m: str(_get(values, m.group(1))), s[2:])
        assert "{{" not in arg, arg
        args.append(arg)
    return args, values


def render_kustomize_args():
    """The kustomize DaemonSet's args with $(VAR) expanded from the ConfigMap and the pod env."""
    docs = {}
    for rel in ("deploy/k8s/daemonset.yaml", "deploy/k8s/configmap.yaml"):
        with open(os.path.join(ROOT, rel)) as fh:
            for d in yaml.safe_load_all(fh):
                if d:
                    docs[d["kind"]] = d
    c = docs["DaemonSet"]["spec"]["template"]["spec"]["containers"][0]
    env = {k: str(v) for k, v in docs["ConfigMap"]["data"].items() if k.isupper()}
    for e in c.get("env", []):
        env[e["name"]] = str(e.get("value", f"<{e['name']}>"))
    out = []
    for a in c["args"]:
        a2 = re.sub(r"\$\((\w+)\)", lambda m: env[m.group(1)], a)
        out.append(a2)
    return out, c


def _check(args):
    from llm_slo_ebpf_toolkit_amd.agent.daemon import Agent, AgentOptions
    from llm_slo_ebpf_toolkit_amd.cli import agent as cli

    opts, smoke = cli.parse(args)
    assert not smoke
    assert isinstance(opts, AgentOptions)
    assert opts.engine == "gpu" and opts.source == "bpf", (opts.engine, opts.source)
    assert opts.gpus == 1  # one worker on one GPU; node-wide multi-GPU fusion is opt-in
    assert opts.model_path.endswith(SHIPPED_MODEL.split("/", 1)[1])
    assert opts.otlp_receiver_bind.endswith(":4318") and opts.otlp_receiver_allow
    a = Agent(AgentOptions(**{**opts.__dict__, "config": os.path.join(ROOT, "config", "toolkit.yaml"),
                              "metrics_bind": "", "output": "stdout"}))
    a.o.model_path = os.path.join(ROOT, SHIPPED_MODEL)
    model, image, meta = a._load_model()  # the model file the image ships loads
    assert meta["name"] == "bayes_learned" and image.size == 9208
    a.close()


def test_helm_chart_args_start_the_agent():
    args, values = render_chart_args()
    assert values["agent"]["source"] == "bpf"
    _check(args)


def test_kustomize_daemonset_args_start_the_agent():
    args, c = render_kustomize_args()
    _check(args)
    names = {e["name"] for e in c.get("env", [])}
    assert "HIP_VISIBLE_DEVICES" not in names  # the worker picks its GPU itself


# measured: the agent with one worker at 1M events/s, profiles/r3_agent_overhead_1Mevs.json (787 MB);
# the HIP runtime's floor per worker process at one hardware queue (docs/BENCHMARKS.md, 465 MB)
AGENT_ONE_WORKER_MB, WORKER_FLOOR_MB, MI355X_NODE_GPUS = 787, 465, 8


def _mib(q: str) -> float:
    q = str(q)
    for suf, f in (("Gi", 1024.0), ("Mi", 1.0), ("G", 1000 ** 3 / 2 ** 20), ("M", 1000 ** 2 / 2 ** 20)):
        if q.endswith(suf):
            return float(q[: -len(suf)]) * f
    return float(q) / 2 ** 20


def _cores(q: str) -> float:
    q = str(q)
    return float(q[:-1]) / 1000 if q.endswith("m") else float(q)


def _sized(gpus: int, limits: dict) -> None:
    workers = gpus if gpus > 0 else MI355X_NODE_GPUS
    need = AGENT_ONE_WORKER_MB + (workers - 1) * WORKER_FLOOR_MB
    assert _mib(limits["memory"]) * 1.048576 >= need, (limits, workers, need)  # MiB -> MB
    assert _cores(limits["cpu"]) >= 0.5 * workers, (limits, workers)


def test_shipped_resources_fit_the_workers_they_start():
    """the memory limit must hold every worker the args start (each carries
    the HIP runtime's resident floor) and the CPU limit must not be shared by N workers."""
    args, values = render_chart_args()
    _sized(int(values["agent"]["gpus"]), values["resources"]["limits"])
    kargs, c = render_kustomize_args()
    g = int(next(a.split("=", 1)[1] for a in kargs if a.startswith("--gpus=")))
    _sized(g, c["resources"]["limits"])


def test_shipped_signal_set_loads_the_gpu_and_cfs_probes():
    """the shipped config enables the GPU signals and CFS throttling, so the
    loader's probe specs include gpu_kfd.bpf.o (and the HIP uprobes in it) and cfs_throttle.bpf.o."""
    from llm_slo_ebpf_toolkit_amd.agent.daemon import choose_enabled_signals
    from llm_slo_ebpf_toolkit_amd.collector import loader
    from llm_slo_ebpf_toolkit_amd.contracts import config as toolkitcfg
    from llm_slo_ebpf_toolkit_amd.signals import catalog

    docs = {}
    with open(os.path.join(ROOT, "deploy/k8s/configmap.yaml")) as fh:
        for d in yaml.safe_load_all(fh):
            docs[d["kind"]] = d
    sets = [yaml.safe_load(docs["ConfigMap"]["data"]["toolkit.yaml"])["signal_set"]]
    with open(os.path.join(ROOT, "charts/llm-slo-agent/values.yaml")) as fh:
        sets.append(yaml.safe_load(fh)["config"]["signal_set"])

    class AllObjects(loader.BpfProbeLoader):
        def available(self):
            return list(loader.PROBE_SIGNALS)

    for sig in sets:
        assert set(catalog.DEPLOY_SIGNALS) <= set(sig), sig
        cfg = toolkitcfg.default()
        cfg.signal_set = sig
        enabled = choose_enabled_signals(cfg.signal_set, [], catalog.supported_signals_for_mode(catalog.MODE_GPU))
        specs = loader.probe_specs(AllObjects("/nonexistent"), enabled)
        loaded = {s.signal for s in specs}
        assert {"gpu_queue_delay_ms", "rccl_collective_ms", "cfs_throttled_ms"} <= loaded, loaded


def test_helm_test_pod_checks_the_agent_endpoints():
    with open(os.path.join(ROOT, "charts/llm-slo-agent/templates/tests/test-connection.yaml")) as fh:
        text = fh.read()
    assert '"helm.sh/hook": test' in text
    for path in ("/healthz", "/readyz", "/metrics"):
        assert path in text
    for name in re.findall(r"\^(llm_slo_agent_\w+)", text):
        from llm_slo_ebpf_toolkit_amd.agent.metrics import AgentMetrics

        m = AgentMetrics("probe", "core_full", [], [])
        assert name in m.registry.exposition(), name


def test_shipped_model_is_what_attributor_train_produces():
    """config/models/mislo-learned.safetensors is `attributor --train` with its defaults: the
    deterministic training set and fit reproduce it, and on REF's 55 rows it beats REF's table
    on all three of REF's quality numbers."""
    from llm_slo_ebpf_toolkit_amd.models import train

    model, image, meta = train.load_model(os.path.join(ROOT, SHIPPED_MODEL))
    tm = train.train_cpu(train.TrainConfig())
    np.testing.assert_array_equal(image, tm.image())
    r = meta["ref55"]
    assert r["single_fault_macro_f1"] >= 0.9818 and r["multi_fault_partial_accuracy"] >= 1.0
    assert r["multi_fault_coverage_accuracy"] >= 0.667


def _mode_env(*args):
    import subprocess

    p = subprocess.run(["bash", os.path.join(ROOT, "scripts/chaos/set_agent_mode.sh"), *args],
                       env=dict(os.environ, DRY_RUN="1"), capture_output=True, text=True)
    return p, dict(ln.split("=", 1) for ln in p.stdout.split())


def test_set_agent_mode_values_start_the_agent():
    """scripts/chaos/set_agent_mode.sh (REF scripts/chaos/set_agent_mode.sh:1-37) sets the env the
    DaemonSet's args read; every mode it accepts -- its defaults included -- must parse with the
    agent's CLI (round 4 defaulted SOURCE=ring, which `agent --source` rejects: crash loop)."""
    from llm_slo_ebpf_toolkit_amd.cli import agent as cli

    for args in ((), ("gpu", "bpf"), ("cpu", "replay", "jsonl", "both"), ("synthetic", "shm", "stdout", "slo")):
        p, env = _mode_env(*args)
        assert p.returncode == 0, p.stderr
        base, c = render_kustomize_args()
        rendered = [re.sub(r"--(engine|source|output|event-kind)=\S*", lambda m: f"--{m.group(1)}=" + env[
            {"engine": "ENGINE", "source": "SOURCE", "output": "OUTPUT", "event-kind": "EVENT_KIND"}[m.group(1)]], a)
            for a in base]
        opts, _ = cli.parse(rendered)
        assert (opts.engine, opts.source, opts.output, opts.event_kind) == (
            env["ENGINE"], env["SOURCE"], env["OUTPUT"], env["EVENT_KIND"])
    p, _ = _mode_env("gpu", "ring")
    assert p.returncode == 2 and "SOURCE must be one of" in p.stderr


def test_config_gpu_block_sets_the_window_engine_and_flags_win():
    from llm_slo_ebpf_toolkit_amd.agent.daemon import AgentOptions, apply_gpu_config
    from llm_slo_ebpf_toolkit_amd.cli import agent as cli
    from llm_slo_ebpf_toolkit_amd.contracts.config import GPUConfig

    gpu = GPUConfig(enabled=True, window_ms=500, max_events_per_window=4096, world_size=2, attribution_model="bayes_gpu")
    o, _ = cli.parse(["--engine=gpu"])
    o2 = apply_gpu_config(o, gpu)
    assert (o2.window_ms, o2.window_events, o2.gpus, o2.model) == (500, 4096, 2, "bayes_gpu")
    o, _ = cli.parse(["--engine=gpu", "--window-ms=1000", "--gpus=1"])
    o2 = apply_gpu_config(o, gpu)
    assert (o2.window_ms, o2.gpus, o2.window_events) == (1000, 1, 4096)
    # a learned model comes from --model-path only
    o2 = apply_gpu_config(cli.parse(["--model-path=x.safetensors"])[0], gpu)
    assert o2.model == AgentOptions().model
    o2 = apply_gpu_config(cli.parse([])[0], GPUConfig(enabled=False))
    assert o2.engine == "synthetic"
    assert apply_gpu_config(cli.parse(["--engine=gpu"])[0], GPUConfig(enabled=False)).engine == "gpu"


def test_shipped_gpu_block_agrees_with_the_flags_the_deployments_pass():
    docs = {}
    with open(os.path.join(ROOT, "deploy/k8s/configmap.yaml")) as fh:
        cm = yaml.safe_load(fh)
    cfg = yaml.safe_load(cm["data"]["toolkit.yaml"])
    assert cfg["gpu"]["world_size"] == int(cm["data"]["GPUS"])
    with open(os.path.join(ROOT, "charts/llm-slo-agent/values.yaml")) as fh:
        values = yaml.safe_load(fh)
    assert values["config"]["gpu"]["world_size"] == values["agent"]["gpus"]
    assert cfg["gpu"]["attribution_model"] in ("bayes", "bayes_gpu")
    assert values["config"]["gpu"]["attribution_model"] in ("bayes", "bayes_gpu")
