#!/usr/bin/env bash
# Fault matrix: for every scenario x rerun, produce the artefacts the M5 gate consumes
# (raw_samples.jsonl + collector_overhead.csv per run directory), attribute the replayed
# incidents and write the benchmark bundle. The incident artefacts are synthetic (faultinject /
# faultreplay); REAL_INJECTORS=true additionally applies tc-netem delay/loss (network scenarios)
# or a CPU burner in the kind nodes while the run's artefacts are produced -- it does not route
# measured signals into them.
#
# collector_overhead.csv (the gate's B5 input) is measured on the agent that ships: the window
# agent (ENGINE=gpu on the MI355X runner, cpu elsewhere) with the ConfigMap's toolkit.yaml, the
# shipped model, the native samplers and the OTLP receiver, at OVERHEAD_RATE events/s for
# OVERHEAD_SECONDS (tools/agent_overhead.py).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
export PYTHONPATH="$ROOT${PYTHONPATH:+:$PYTHONPATH}"
CLI="python3 -m llm_slo_ebpf_toolkit_amd.cli"
OUT=${OUT:-$ROOT/artifacts/weekly-benchmark}
SCENARIOS=${SCENARIOS:-"dns_latency cpu_throttle provider_throttle memory_pressure network_partition mixed mixed_multi"}
RUNS=${RUNS:-3}
COUNT=${COUNT:-36}
REAL_INJECTORS=${REAL_INJECTORS:-false}
if [ -e /dev/kfd ]; then ENGINE=${ENGINE:-gpu}; else ENGINE=${ENGINE:-cpu}; fi
OVERHEAD_RATE=${OVERHEAD_RATE:-1e6}
OVERHEAD_SECONDS=${OVERHEAD_SECONDS:-10}

inject_real() {  # $1 scenario, $2 on|off
  local node=${KIND_NODE:-llm-slo-lab-worker}
  case "$1" in
    dns_latency|network_partition)
      if [ "$2" = on ]; then docker exec "$node" tc qdisc add dev eth0 root netem delay 200ms loss 2% || true
      else docker exec "$node" tc qdisc del dev eth0 root || true; fi ;;
    cpu_throttle)
      if [ "$2" = on ]; then kubectl run cpu-burner --image=busybox --restart=Never -- sh -c 'while :; do :; done' || true
      else kubectl delete pod cpu-burner --ignore-not-found; fi ;;
  esac
}

for sc in $SCENARIOS; do
  for run in $(seq 1 "$RUNS"); do
    dir="$OUT/$sc/run-$run"
    mkdir -p "$dir"
    [ "$REAL_INJECTORS" = true ] && inject_real "$sc" on
    $CLI.faultinject --scenario "$sc" --count "$COUNT" --out "$dir/raw_samples.jsonl"
    $CLI.faultreplay --scenario "$sc" --count "$COUNT" --with-signals --seed "$run" --out "$dir/fault_samples.jsonl"
    $CLI.attributor --input "$dir/fault_samples.jsonl" --out "$dir/attributions.jsonl" \
      --summary-out "$dir/attribution_summary.json" --confusion-out "$dir/confusion.csv"
    rm -f "$dir/collector_overhead.csv"
    python3 "$ROOT/tools/agent_overhead.py" --engine "$ENGINE" --rate "$OVERHEAD_RATE" \
      --seconds "$OVERHEAD_SECONDS" --warmup 3 --node "${NODE_NAME:-node-a}" \
      --csv "$dir/collector_overhead.csv" --out "$dir/agent_overhead.json" > "$dir/agent_overhead.log" 2>&1
    [ "$REAL_INJECTORS" = true ] && inject_real "$sc" off
  done
done
$CLI.benchgen --out "$OUT/bundle" --scenario mixed_faults
echo "fault matrix written to $OUT"
