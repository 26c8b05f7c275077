#!/usr/bin/env bash
# Drive traffic at the demo service and capture an evidence report from Prometheus.
set -euo pipefail
API=${API:-http://127.0.0.1:8080}
PROM=${PROM:-http://127.0.0.1:9090}
N=${N:-60}
OUT=${OUT:-artifacts/evidence/report.md}
mkdir -p "$(dirname "$OUT")"
for i in $(seq 1 "$N"); do
  curl -s -X POST "$API/chat" -H 'Content-Type: application/json' \
    -d "{\"prompt\":\"evidence run $i\",\"profile\":\"rag_medium\",\"max_tokens\":16,\"request_id\":\"ev-$i\"}" >/dev/null || true
done
q() { curl -s --get "$PROM/api/v1/query" --data-urlencode "query=$1" | python3 -c \
  'import json,sys; r=json.load(sys.stdin)["data"]["result"]; print(r[0]["value"][1] if r else "n/a")'; }
{
  echo "# Evidence report ($(date -u +%Y-%m-%dT%H:%M:%SZ))"
  echo
  echo "| query | value |"
  echo "|---|---|"
  echo "| TTFT p95 (ms) | $(q 'histogram_quantile(0.95, sum(rate(llm_slo_ttft_ms_bucket[5m])) by (le))') |"
  echo "| kernel DNS p95 (ms) | $(q 'histogram_quantile(0.95, sum(rate(llm_ebpf_dns_latency_ms_bucket[5m])) by (le))') |"
  echo "| enrichment ratio | $(q 'sum(rate(llm_slo_correlation_total{enriched="true"}[5m])) / sum(rate(llm_slo_correlation_total[5m]))') |"
  echo "| GPU engine events/s | $(q 'sum(rate(llm_slo_agent_gpu_window_events_total[1m]))') |"
  echo "| agent CPU overhead % | $(q 'max(llm_slo_agent_cpu_overhead_pct)') |"
} > "$OUT"
cat "$OUT"
