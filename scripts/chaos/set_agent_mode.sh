#!/usr/bin/env bash
# Switch the agent DaemonSet between engines / sources / outputs without editing manifests: sets
# the DaemonSet env its args read ($(ENGINE), $(SOURCE), $(OUTPUT), $(EVENT_KIND)), then waits
# for the rollout. Values are checked against the agent's own choices before anything changes.
#   usage: set_agent_mode.sh [gpu|cpu|synthetic] [bpf|shm|replay] [stdout|jsonl|otlp] [probe|slo|both]
#   DRY_RUN=1: print the env assignments, touch nothing (tests/test_deploy_args.py feeds them to
#   the agent's CLI)
set -euo pipefail
NS=${NS:-llm-slo-system}
ENGINE=${1:-gpu}
SOURCE=${2:-bpf}
OUTPUT=${3:-otlp}
EVENT_KIND=${4:-probe}
check() {  # name value allowed...
  local name=$1 v=$2
  shift 2
  for ok in "$@"; do [ "$v" = "$ok" ] && return 0; done
  echo "set_agent_mode: $name must be one of: $* (got '$v')" >&2
  exit 2
}
check ENGINE "$ENGINE" gpu cpu synthetic
check SOURCE "$SOURCE" bpf shm replay
check OUTPUT "$OUTPUT" stdout jsonl otlp
check EVENT_KIND "$EVENT_KIND" probe slo both
if [ "${DRY_RUN:-0}" = "1" ]; then
  printf 'ENGINE=%s\nSOURCE=%s\nOUTPUT=%s\nEVENT_KIND=%s\n' "$ENGINE" "$SOURCE" "$OUTPUT" "$EVENT_KIND"
  exit 0
fi
kubectl -n "$NS" set env daemonset/llm-slo-agent ENGINE="$ENGINE" SOURCE="$SOURCE" OUTPUT="$OUTPUT" \
  EVENT_KIND="$EVENT_KIND"
kubectl -n "$NS" rollout status daemonset/llm-slo-agent --timeout=180s
