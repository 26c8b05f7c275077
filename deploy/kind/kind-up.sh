#!/usr/bin/env bash
# Create the kind lab and deploy observability + agent (synthetic engine, no GPU).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
kind create cluster --config "$ROOT/deploy/kind/kind-config.yaml"
kubectl apply -k "$ROOT/deploy/observability"
kubectl apply -k "$ROOT/deploy/k8s"
kubectl -n llm-slo-system set env daemonset/llm-slo-agent ENGINE=synthetic SOURCE=replay
kubectl -n llm-slo-system rollout status daemonset/llm-slo-agent --timeout=180s
