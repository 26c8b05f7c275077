#!/usr/bin/env bash
# Switch the agent DaemonSet between engines / sources / outputs without editing manifests.
# usage: set_agent_mode.sh [gpu|synthetic] [ring|replay] [stdout|jsonl|otlp] [probe|slo|both]
set -euo pipefail
NS=${NS:-llm-slo-system}
kubectl -n "$NS" set env daemonset/llm-slo-agent ENGINE="${1:-gpu}" SOURCE="${2:-ring}" OUTPUT="${3:-otlp}" \
  EVENT_KIND="${4:-probe}"
kubectl -n "$NS" rollout status daemonset/llm-slo-agent --timeout=180s
