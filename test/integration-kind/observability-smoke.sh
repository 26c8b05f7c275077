#!/usr/bin/env bash
# Observability stack smoke (REF test/integration-kind/observability-smoke.sh): Prometheus,
# Grafana, the OpenTelemetry collector and Tempo roll out; Prometheus scrapes the agent, the
# alert rules load, the collector accepts an OTLP log record (the agent's IncidentAttribution
# export path) and Grafana has the toolkit dashboards provisioned.
set -euo pipefail

ROOT_DIR="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
if ! command -v kind >/dev/null 2>&1 || ! command -v kubectl >/dev/null 2>&1; then
  echo "observability smoke skipped: kind / kubectl not installed"
  exit 0
fi
cd "$ROOT_DIR"
NS=observability
make observability-up
for d in prometheus grafana otel-collector tempo; do
  kubectl -n "$NS" rollout status "deployment/$d" --timeout=300s
done

prom() {  # GET on the Prometheus API through the apiserver proxy
  kubectl get --raw "/api/v1/namespaces/${NS}/services/prometheus:9090/proxy$1"
}
for i in $(seq 1 30); do
  UP="$(prom '/api/v1/query?query=up%7Bjob%3D~%22.*llm-slo.*%22%7D' || true)"
  grep -q '"value"' <<<"$UP" && break
  sleep 10
done
grep -q '"value"' <<<"$UP" || { echo "prometheus is not scraping the agent"; exit 1; }
RULES="$(prom '/api/v1/rules')"
grep -q 'TTFTBudgetBurning' <<<"$RULES" || { echo "toolkit alert rules not loaded"; exit 1; }

# one OTLP/HTTP JSON log record into the collector (the agent's --output=otlp path)
kubectl -n "$NS" run otlp-probe --rm -i --restart=Never --image=curlimages/curl:8.8.0 -- \
  curl -sf -XPOST -H 'Content-Type: application/json' \
  "http://otel-collector.${NS}.svc:4318/v1/logs" \
  -d '{"resourceLogs":[{"resource":{"attributes":[{"key":"service.name","value":{"stringValue":"smoke"}}]},"scopeLogs":[{"logRecords":[{"body":{"stringValue":"smoke"}}]}]}]}' \
  >/dev/null || { echo "otel collector rejected OTLP logs"; exit 1; }

DASH="$(kubectl get --raw "/api/v1/namespaces/${NS}/services/grafana:3000/proxy/api/search?query=" || true)"
grep -qi 'llm' <<<"$DASH" || { echo "grafana dashboards not provisioned"; exit 1; }
echo "observability smoke ok"
