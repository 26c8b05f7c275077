#!/usr/bin/env bash
# Fault matrix: for every scenario x rerun, produce the artefacts the M5 gate consumes
# (raw_samples.jsonl + collector_overhead.csv per run directory), attribute the replayed
# incidents and write the benchmark bundle. Synthetic by default; REAL_INJECTORS=true also
# applies tc-netem delay/loss (network scenarios) or a CPU burner in the kind nodes, in
# which case the agent's measured signals feed the same pipeline.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
export PYTHONPATH="$ROOT${PYTHONPATH:+:$PYTHONPATH}"
CLI="python3 -m llm_slo_ebpf_toolkit_amd.cli"
OUT=${OUT:-$ROOT/artifacts/weekly-benchmark}
SCENARIOS=${SCENARIOS:-"dns_latency cpu_throttle provider_throttle memory_pressure network_partition mixed mixed_multi"}
RUNS=${RUNS:-3}
COUNT=${COUNT:-36}
REAL_INJECTORS=${REAL_INJECTORS:-false}

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
    python3 - "$dir" <<'PY'
import csv, os, sys
from llm_slo_ebpf_toolkit_amd.evaluation import overhead
d = sys.argv[1]
m = overhead.measure(duration_s=1.0, mode="agent")
with open(os.path.join(d, "collector_overhead.csv"), "w", newline="") as fh:
    w = csv.writer(fh)
    w.writerow(["timestamp", "node", "collector_cpu_pct", "collector_memory_mb", "events_per_second", "dropped_events"])
    w.writerow([m.get("timestamp", ""), os.environ.get("NODE_NAME", "node-a"), f"{m['cpu_pct']:.4f}",
                f"{m.get('rss_mb', 0):.1f}", f"{m.get('events_per_second', 0):.1f}", 0])
PY
    [ "$REAL_INJECTORS" = true ] && inject_real "$sc" off
  done
done
$CLI.benchgen --out "$OUT/bundle" --scenario mixed_faults
echo "fault matrix written to $OUT"
