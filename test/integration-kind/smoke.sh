#!/usr/bin/env bash
# kind integration smoke (REF test/integration-kind/smoke.sh): the agent DaemonSet rolls out
# on a kind cluster (no GPU there: the synthetic engine, REF's tick loop) and serves its
# metrics; the demo RAG service rolls out and answers a chat request. On an MI355X node pool
# the same manifests run the GPU engine (deploy/k8s, ENGINE=gpu in the ConfigMap).
set -euo pipefail

ROOT_DIR="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"

if [[ "$(uname -s | tr '[:upper:]' '[:lower:]')" != "linux" ]]; then
  echo "kind integration smoke skipped: linux required"
  exit 0
fi
if ! command -v kind >/dev/null 2>&1 || ! command -v kubectl >/dev/null 2>&1; then
  echo "kind integration smoke skipped: kind / kubectl not installed"
  exit 0
fi

cd "$ROOT_DIR"
make kind-up
kubectl apply -k deploy/k8s
# kind nodes have no /dev/kfd: run the REF synthetic tick loop there
kubectl -n llm-slo-system set env daemonset/llm-slo-agent ENGINE=synthetic SOURCE=replay
kubectl -n llm-slo-system rollout status daemonset/llm-slo-agent --timeout=240s

AGENT_POD="$(kubectl -n llm-slo-system get pods -l app.kubernetes.io/name=llm-slo-agent \
  -o jsonpath='{.items[0].metadata.name}')"
[[ -n "$AGENT_POD" ]] || { echo "failed to resolve agent pod"; exit 1; }

METRICS="$(kubectl get --raw "/api/v1/namespaces/llm-slo-system/pods/${AGENT_POD}:2112/proxy/metrics")"
grep -q 'llm_slo_agent_up 1' <<<"$METRICS" || { echo "agent not up"; exit 1; }
grep -q 'llm_slo_agent_event_kind{kind="probe"} 1' <<<"$METRICS" || { echo "expected probe mode metric"; exit 1; }
grep -q 'llm_slo_agent_signal_enabled' <<<"$METRICS" || { echo "expected signal toggle metrics"; exit 1; }
grep -q 'llm_slo_agent_memory_rss_bytes' <<<"$METRICS" || { echo "expected the agent RSS gauge"; exit 1; }

kubectl apply -k deploy/demo/rag-service
kubectl rollout status deployment/rag-service --timeout=240s
RAG_POD="$(kubectl get pods -l app=rag-service -o jsonpath='{.items[0].metadata.name}')"
OUT="$(kubectl exec "$RAG_POD" -- python3 -c '
import json, urllib.request
req = urllib.request.Request("http://127.0.0.1:8080/chat", data=json.dumps({"prompt": "kind smoke"}).encode(),
                             headers={"Content-Type": "application/json"}, method="POST")
print(urllib.request.urlopen(req, timeout=30).read().decode())')"
grep -q '"trace_id"' <<<"$OUT" || { echo "rag-service chat failed: $OUT"; exit 1; }
echo "kind smoke ok"
