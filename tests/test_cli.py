"""Every CLI (REF cmd/*, which REF leaves untested) run in-process with REF flags."""

import csv
import json
import os

import pytest

from llm_slo_ebpf_toolkit_amd.cli import agent, attributor, benchgen, collector, correlationeval, faultinject, \
    faultreplay, loadgen, m5gate, schemavalidate, sloctl
from llm_slo_ebpf_toolkit_amd.contracts import validator

from conftest import FIXTURES, ROOT


def read_jsonl(path):
    with open(path) as fh:
        return [json.loads(x) for x in fh if x.strip()]


@pytest.mark.parametrize("mod", [agent, attributor, benchgen, collector, correlationeval, faultinject, faultreplay,
                                 loadgen, m5gate, schemavalidate, sloctl])
def test_version(mod, capsys):
    assert mod.main(["--version"]) == 0
    assert capsys.readouterr().out.strip()


def test_faultreplay_and_attributor(tmp_path):
    fx = tmp_path / "fs.jsonl"
    assert faultreplay.main(["--scenario", "mixed", "--count", "14", "--out", str(fx), "--with-signals"]) == 0
    out, summ, conf = tmp_path / "a.jsonl", tmp_path / "s.json", tmp_path / "c.csv"
    assert attributor.main(["-input", str(fx), "-out", str(out), "--summary-out", str(summ), "--confusion-out",
                            str(conf), "--config", str(tmp_path / "missing.yaml")]) == 0
    rows = read_jsonl(out)
    assert len(rows) == 14
    for r in rows:
        validator.validate("incident-attribution", r)
    s = json.load(open(summ))
    # with profile signals REF's table confuses provider_throttle/provider_error (the mf-04 effect)
    assert s["total_samples"] == 14 and s["attribution_mode"] == "bayes" and s["accuracy"] >= 0.8
    with open(conf) as fh:
        assert next(csv.reader(fh)) == ["actual", "predicted", "count"]


def test_attributor_ref_dataset_macro_f1(tmp_path):
    summ = tmp_path / "s.json"
    assert attributor.main(["--input", os.path.join(FIXTURES, "ref_multi_fault_samples.jsonl"), "--out",
                            str(tmp_path / "o.jsonl"), "--summary-out", str(summ)]) == 0
    s = json.load(open(summ))
    assert s["accuracy"] == pytest.approx(0.5273, abs=1e-4)
    assert s["single_fault_macro_f1"] == pytest.approx(0.9818, abs=1e-4)
    assert s["partial_accuracy"] == pytest.approx(0.9818, abs=1e-4)


def test_attributor_bayes_learned_defaults_to_the_shipped_model(tmp_path):
    """`attributor --attribution-mode bayes_learned` without --model-path scores with the shipped
    trained model (config/models/mislo-learned.safetensors), as the DaemonSet's agent does."""
    summ = tmp_path / "s.json"
    rc = attributor.main(["--attribution-mode", "bayes_learned", "--input", os.path.join(FIXTURES, "ref_multi_fault_samples.jsonl"),
                          "--out", str(tmp_path / "a.jsonl"), "--summary-out", str(summ)])
    assert rc == 0
    s = json.loads(summ.read_text())
    assert s["attribution_mode"] == "model:mislo-learned.safetensors" and s["single_fault_macro_f1"] == 1.0


def test_attributor_default_sample_rule_mode(capsys):
    assert attributor.main(["--attribution-mode", "rule"]) == 0
    row = json.loads(capsys.readouterr().out.strip())
    assert row["predicted_fault_domain"] == "provider_throttle"


def test_attributor_webhook_strict_failure(tmp_path, http_recorder):
    srv = http_recorder([(400, "no")])
    rc = attributor.main(["--out", str(tmp_path / "o.jsonl"), "--webhook-enabled", "--webhook-url", srv.url,
                          "--webhook-strict"])
    assert rc == 1 and len(srv.requests) == 1
    assert attributor.main(["--out", str(tmp_path / "o.jsonl"), "--webhook-enabled", "--webhook-url", srv.url,
                            "--webhook-format", "bogus"]) == 2


def test_faultinject_and_collector(tmp_path):
    raw = tmp_path / "raw.jsonl"
    assert faultinject.main(["--scenario", "mixed", "--count", "6", "--out", str(raw)]) == 0
    assert len(read_jsonl(raw)) == 6
    out = tmp_path / "ev.jsonl"
    assert collector.main(["--input", str(raw), "--output", "jsonl", "--output-path", str(out)]) == 0
    evs = read_jsonl(out)
    assert len(evs) == 24
    for e in evs:
        validator.validate("slo-event", e)


def test_collector_synthetic_otlp(http_recorder, tmp_path):
    srv = http_recorder()
    empty = tmp_path / "empty.jsonl"
    empty.write_text("")
    assert collector.main(["--input", str(empty), "--output", "otlp", "--otlp-endpoint", srv.url + "/v1/logs",
                           "--count", "3", "--scenario", "dns_latency"]) == 0
    n = sum(len(json.loads(r["body"])["resourceLogs"][0]["scopeLogs"][0]["logRecords"]) for r in srv.requests)
    assert n == 12


def test_collector_bad_output_mode(tmp_path):
    empty = tmp_path / "empty.jsonl"
    empty.write_text("")
    assert collector.main(["--input", str(empty), "--output", "carrier"]) == 1


def test_benchgen(tmp_path):
    assert benchgen.main(["--out", str(tmp_path / "b"), "--scenario", "mixed_faults", "--measure-seconds", "0.2"]) == 0
    files = set(os.listdir(tmp_path / "b"))
    for f in ("attribution_summary.json", "collector_overhead.csv", "confusion-matrix.csv"):
        assert f in files, files


def test_correlationeval(tmp_path):
    out, pred = tmp_path / "s.json", tmp_path / "p.csv"
    assert correlationeval.main(["--input", os.path.join(FIXTURES, "ref_labeled_pairs.jsonl"), "--out", str(out),
                                 "--predictions-out", str(pred)]) == 0
    s = json.load(open(out))
    assert s["precision"] == 1.0 and s["recall"] == 1.0 and s["sample_size"] == 55 and s["passed_gate"]
    with open(pred) as fh:
        rows = list(csv.reader(fh))
    assert rows[0][0] == "case_id" and len(rows) == 56
    assert correlationeval.main(["--input", os.path.join(FIXTURES, "ref_labeled_pairs.jsonl"), "--out", str(out),
                                 "--predictions-out", str(pred), "--min-precision", "1.01"]) == 1


def test_m5gate(tmp_path):
    from test_releasegate import populate

    cand, base = populate(tmp_path)
    js, md = tmp_path / "g.json", tmp_path / "g.md"
    assert m5gate.main(["--candidate-root", cand, "--baseline-root", base, "--scenarios", "dns_latency",
                        "--out-json", str(js), "--out-md", str(md)]) == 0
    assert json.load(open(js))["pass"] and "M5 Gate Summary" in md.read_text()
    assert m5gate.main(["--candidate-root", cand, "--baseline-root", base, "--scenarios", "dns_latency",
                        "--max-overhead-pct", "1", "--out-json", str(js), "--out-md", str(md)]) == 1


def test_loadgen(tmp_path):
    out = tmp_path / "req.jsonl"
    assert loadgen.main(["--profile", "chat_short", "--duration-sec", "2", "--rps", "5", "--out", str(out)]) == 0
    rows = read_jsonl(out)
    assert len(rows) == 10 and rows[3]["request_id"] == "req-000003"
    assert all(r["prompt_class"] == "chat_short" and 80 <= r["expected_ttft_ms"] < 150 for r in rows)
    assert all(2 <= r["retrieval_docs"] <= 9 and 64 <= r["target_tokens"] < 576 for r in rows)
    assert loadgen.main(["--rps", "0", "--out", str(out)]) == 1


def test_schemavalidate(capsys, monkeypatch):
    monkeypatch.chdir(ROOT)
    assert schemavalidate.main([]) == 0
    assert capsys.readouterr().out.count("ok:") == 4


def test_sloctl(capsys, http_recorder):
    assert sloctl.main([]) == 2
    assert sloctl.main(["bogus"]) == 2
    capsys.readouterr()
    rc = sloctl.main(["prereq", "check", "--output", "json"])
    rep = json.loads(capsys.readouterr().out)
    assert rc in (0, 1) and {c["name"] for c in rep["checks"]} >= {"host_linux", "gpu_gfx950", "rccl_library"}
    ok = json.dumps({"status": "success", "data": {"resultType": "vector", "result": [{"value": [1, "0.01"]}]}})
    srv = http_recorder([(200, ok)] * 3)
    assert sloctl.main(["cdgate", "check", "--prometheus-url", srv.url, "--output", "json"]) == 0
    srv2 = http_recorder([(500, "x")])
    assert sloctl.main(["cdgate", "check", "--prometheus-url", srv2.url, "--fail-open=false"]) == 1
    srv3 = http_recorder([(500, "x")])
    assert sloctl.main(["cdgate", "check", "--prometheus-url", srv3.url, "--fail-open"]) == 0


def test_agent_synthetic_count(tmp_path):
    out = tmp_path / "agent.jsonl"
    assert agent.main(["--count", "3", "--event-kind", "both", "--output", "jsonl", "--output-path", str(out),
                       "--metrics-bind", "", "--scenario", "dns_latency", "--disable-overhead-guard", "--config",
                       os.path.join(ROOT, "config", "toolkit.yaml")]) == 0
    rows = read_jsonl(out)
    slo = [r for r in rows if "sli_name" in r]
    probe = [r for r in rows if "signal" in r]
    assert len(slo) == 12 and len(probe) == 3 * 9
    assert agent.main(["--event-kind", "weird", "--metrics-bind", ""]) == 1


def test_agent_metrics_export_gpu_signal_histograms():
    import numpy as np

    from llm_slo_ebpf_toolkit_amd.agent.metrics import AgentMetrics
    from llm_slo_ebpf_toolkit_amd.signals import catalog

    m = AgentMetrics("both", "gpu", catalog.SIGNAL_NAMES, catalog.SIGNAL_NAMES)
    hist = np.zeros((16, 16), dtype=np.uint32)
    slot = catalog.BY_NAME["gpu_queue_delay_ms"].slot
    hist[slot, 2] = 7  # le 5 ms
    sums = np.zeros(16, dtype=np.int64)
    sums[slot] = 7 * 4000  # 7 x 4 ms, in 1/1000 ms
    m.observe_window(hist, np.zeros((16, 3), dtype=np.uint32), np.zeros(8, dtype=np.int64), 7, 1.0, "n", "p", "ns",
                     value_sums_milli=sums)
    text = m.registry.exposition() if hasattr(m, "registry") else m.r.exposition()
    assert 'llm_ebpf_gpu_queue_delay_ms_bucket{le="5"} 7' in text
    assert "llm_ebpf_gpu_queue_delay_ms_sum 28" in text


def test_agent_metrics_export_otlp_outcomes_and_memory_charge():
    from types import SimpleNamespace

    from llm_slo_ebpf_toolkit_amd.agent.metrics import AgentMetrics
    from llm_slo_ebpf_toolkit_amd.signals import catalog

    m = AgentMetrics("both", "gpu", catalog.SIGNAL_NAMES, catalog.SIGNAL_NAMES)
    m.set_otlp(SimpleNamespace(accepted=40, dropped=2, rejected=1),
               SimpleNamespace(conflicts=3, spoofed=0, early_dropped=5))
    m.set_rss()
    text = m.registry.exposition() if hasattr(m, "registry") else m.r.exposition()
    for outcome, v in (("accepted", 40), ("dropped", 2), ("rejected", 1), ("conflict", 3), ("first_token_late", 5)):
        assert f'llm_slo_agent_otlp_spans{{outcome="{outcome}"}} {v}' in text, outcome
    assert "llm_slo_agent_memory_rss_bytes" in text and "llm_slo_agent_memory_cgroup_bytes" in text


def test_agent_gpu_hw_queues_flag_wins_over_env_default_does_not(monkeypatch):
    from llm_slo_ebpf_toolkit_amd.cli import agent as agent_cli

    for k in ("MISLO_ONE_STREAM", "HSA_ENABLE_SDMA"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")  # a node-wide setting
    agent_cli.parse(["--engine", "gpu"])
    assert os.environ["GPU_MAX_HW_QUEUES"] == "4"
    agent_cli.parse(["--engine", "gpu", "--gpu-hw-queues", "1"])
    assert os.environ["GPU_MAX_HW_QUEUES"] == "1"
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    agent_cli.parse(["-gpu-hw-queues=2"])
    assert os.environ["GPU_MAX_HW_QUEUES"] == "2"
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    monkeypatch.delenv("MISLO_ONE_STREAM", raising=False)
    monkeypatch.delenv("HSA_ENABLE_SDMA", raising=False)
    agent_cli.parse([])
    assert os.environ["GPU_MAX_HW_QUEUES"] == "1"
    # one hardware queue: one HIP stream and blit-kernel copies (no SDMA queue save area)
    assert os.environ["MISLO_ONE_STREAM"] == "1" and os.environ["HSA_ENABLE_SDMA"] == "0"


def test_agent_keeps_two_streams_and_sdma_with_more_hardware_queues(monkeypatch):
    from llm_slo_ebpf_toolkit_amd.cli import agent as agent_cli

    for k in ("GPU_MAX_HW_QUEUES", "MISLO_ONE_STREAM", "HSA_ENABLE_SDMA"):
        monkeypatch.delenv(k, raising=False)
    agent_cli.parse(["--gpu-hw-queues", "4"])
    assert os.environ["GPU_MAX_HW_QUEUES"] == "4"
    assert "MISLO_ONE_STREAM" not in os.environ and "HSA_ENABLE_SDMA" not in os.environ
    monkeypatch.setenv("HSA_ENABLE_SDMA", "1")  # an operator's explicit setting wins
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    agent_cli.parse([])
    assert os.environ["HSA_ENABLE_SDMA"] == "1"


# REF's flag surface per binary (cmd/agent/main.go:334-373, cmd/collector/main.go:25-41,
# cmd/attributor/main.go:53-69, cmd/m5gate/main.go:22-39): every flag is accepted and documented
REF_FLAGS = {
    agent: "--cluster --namespace --workload --service --k8s-node --pod --container --scenario --count --interval-ms "
           "--event-kind --output --output-path --otlp-endpoint --otlp-timeout-ms --webhook-url --webhook-secret "
           "--webhook-format --webhook-timeout-ms --capability-mode --disable-signals --disable-overhead-guard "
           "--config --enable-hello-tracer --hello-target-comm --enable-real-probe-metrics --metrics-bind --probe-smoke",
    collector: "--input --output --output-path --otlp-endpoint --otlp-timeout-ms --cluster --namespace --workload "
               "--service --k8s-node --scenario --count --interval-ms",
    attributor: "--input --out --summary-out --confusion-out --schema --config --attribution-mode --webhook-enabled "
                "--webhook-url --webhook-secret --webhook-format --webhook-timeout-ms --webhook-strict",
    benchgen: "--out --scenario --workload --input --attribution-mode",
    faultreplay: "--scenario --count --out",
    faultinject: "--scenario --count --out --cluster --namespace --workload --service --node",
    correlationeval: "--input --out --predictions-out --window-ms --threshold --min-precision --min-recall",
    m5gate: "--candidate-root --baseline-root --baseline-manifest --candidate-ref --candidate-commit "
            "--require-baseline-manifest --scenarios --max-overhead-pct --max-variance-pct --min-runs "
            "--ttft-regression-pct --alpha --bootstrap-iters --seed --min-samples --min-cliffs-delta --out-json --out-md",
    loadgen: "--profile --duration-sec --rps --seed --out",
}


@pytest.mark.parametrize("mod", list(REF_FLAGS), ids=lambda m: m.__name__.rsplit(".", 1)[-1])
def test_help_lists_refs_flags(mod, capsys):
    """`--help` renders (a '%' in a help string once broke the agent's) and names REF's flags."""
    with pytest.raises(SystemExit) as e:
        mod.main(["--help"])
    assert e.value.code == 0
    out = capsys.readouterr().out
    assert [f for f in REF_FLAGS[mod].split() if f not in out] == []
