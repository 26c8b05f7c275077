#!/usr/bin/env bash
# Privileged smoke: BPF map creation through bpf(2) (agent --probe-smoke) and, when the
# objects were built (make ebpf-gen) and bpftool exists, a verifier load of every object.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
export PYTHONPATH="$ROOT${PYTHONPATH:+:$PYTHONPATH}"
python3 -m llm_slo_ebpf_toolkit_amd.cli.agent --probe-smoke
OBJ="$ROOT/llm_slo_ebpf_toolkit_amd/probes/ebpf/build"
if command -v bpftool >/dev/null && [ -d "$OBJ" ]; then
  for o in "$OBJ"/*.bpf.o; do
    pin="/sys/fs/bpf/mislo_smoke_$(basename "$o" .bpf.o)"
    bpftool prog loadall "$o" "$pin" && rm -rf "$pin"
    echo "verifier ok: $(basename "$o")"
  done
else
  echo "bpftool or built objects missing: map-creation smoke only"
fi
