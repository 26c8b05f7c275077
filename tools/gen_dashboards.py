"""Generate the Grafana dashboards (dashboards/*.json) from one panel table, so every
query references metrics the agent / demo actually export (checked by tests)."""

import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DASHBOARDS = {
    "slo-overview": ("LLM SLO overview", [
        ("TTFT p95 (ms)", "histogram_quantile(0.95, sum(rate(llm_slo_ttft_ms_bucket[5m])) by (le))", "timeseries"),
        ("Tokens/s p50", "histogram_quantile(0.5, sum(rate(llm_slo_tokens_per_sec_bucket[5m])) by (le))",
         "timeseries"),
        ("Error rate", "sum(rate(llm_slo_errors_total[5m])) / clamp_min(sum(rate(llm_slo_requests_total[5m])), 1e-9)",
         "timeseries"),
        ("Burn rate", "max(llm_slo_burn_rate)", "stat"),
        ("Requests by status", "sum by (status) (rate(llm_slo_requests_total[5m]))", "timeseries"),
    ]),
    "kernel-correlation": ("Kernel signal correlation", [
        ("DNS latency p95 (kernel)", "histogram_quantile(0.95, sum(rate(llm_ebpf_dns_latency_ms_bucket[5m])) by (le))",
         "timeseries"),
        ("Probe events by signal/status", "sum by (signal, status) (rate(llm_ebpf_probe_events_total[5m]))",
         "timeseries"),
        ("Correlation tiers", "sum by (tier, enriched) (rate(llm_slo_correlation_total[5m]))", "timeseries"),
        ("Join outcomes (GPU)", "sum by (outcome) (rate(llm_slo_agent_correlation_pairs_total[5m]))", "timeseries"),
        ("Retrieval DNS (ms) p95", "histogram_quantile(0.95, sum(rate(llm_slo_retrieval_dns_ms_bucket[5m])) by (le))",
         "timeseries"),
    ]),
    "incident-lab": ("Incident lab", [
        ("Attributions by domain", "sum by (domain) (rate(llm_slo_agent_attributions_total[5m]))", "timeseries"),
        ("Signals enabled", "sum by (signal) (llm_slo_agent_signal_enabled)", "table"),
        ("Dropped events", "sum by (reason) (rate(llm_slo_agent_dropped_events_total[5m]))", "timeseries"),
        ("Capability mode", "max by (mode) (llm_slo_agent_capability_mode)", "table"),
    ]),
    "evidence-e2e": ("Evidence end-to-end", [
        ("Agent up", "min(llm_slo_agent_up)", "stat"),
        ("Heartbeat age (s)", "time() - max(llm_slo_agent_heartbeat)", "stat"),
        ("Agent CPU overhead %", "max by (instance) (llm_slo_agent_cpu_overhead_pct)", "timeseries"),
        ("Hello syscalls", "sum by (comm) (rate(llm_ebpf_hello_syscalls_total[5m]))", "timeseries"),
        ("Event kind", "max by (kind) (llm_slo_agent_event_kind)", "table"),
    ]),
    "gpu-engine": ("MI355X window engine", [
        ("Events/s through the GPU engine", "sum(rate(llm_slo_agent_gpu_window_events_total[1m]))", "timeseries"),
        ("Window latency p95 (ms)",
         "histogram_quantile(0.95, sum(rate(llm_slo_agent_gpu_window_latency_ms_bucket[5m])) by (le))", "timeseries"),
        ("Windows/s", "sum(rate(llm_slo_agent_gpu_windows_total[1m]))", "timeseries"),
        ("GPU signals by status",
         'sum by (signal, status) (rate(llm_ebpf_probe_events_total{signal=~"gpu_.*|hbm_.*|xgmi_.*|rccl_.*"}[5m]))',
         "timeseries"),
        ("Ring drops", "max by (instance) (llm_slo_agent_ring_dropped_events)", "stat"),
    ]),
}


def dashboard(uid: str, title: str, panels):
    out = []
    for i, (ptitle, expr, kind) in enumerate(panels):
        out.append({"id": i + 1, "title": ptitle, "type": kind, "datasource": {"type": "prometheus", "uid": "Prometheus"},
                    "gridPos": {"h": 8, "w": 12, "x": (i % 2) * 12, "y": (i // 2) * 8},
                    "targets": [{"refId": "A", "expr": expr}]})
    return {"uid": uid, "title": title, "schemaVersion": 39, "version": 1, "time": {"from": "now-1h", "to": "now"},
            "refresh": "30s", "tags": ["llm-slo", "mi355x"], "panels": out}


def main():
    d = os.path.join(ROOT, "dashboards")
    os.makedirs(d, exist_ok=True)
    for uid, (title, panels) in DASHBOARDS.items():
        with open(os.path.join(d, uid + ".json"), "w") as fh:
            json.dump(dashboard(uid, title, panels), fh, indent=2)
            fh.write("\n")
        print("wrote", uid)


if __name__ == "__main__":
    main()
