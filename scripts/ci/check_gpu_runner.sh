#!/usr/bin/env bash
# Exit 0 when this runner can run the MI355X jobs (gfx950 visible through KFD, ROCm installed).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
export PYTHONPATH="$ROOT${PYTHONPATH:+:$PYTHONPATH}"
python3 -m llm_slo_ebpf_toolkit_amd.cli.sloctl prereq check --require-gpu --output json > /tmp/prereq.json || true
python3 - <<'PY'
import json, sys
r = json.load(open("/tmp/prereq.json"))
need = {c["name"]: c["pass"] for c in r["checks"]}
ok = need.get("gpu_gfx950") and need.get("rocm_installed") and need.get("amdgpu_kfd")
print("gpu runner:", "ready" if ok else "not ready")
sys.exit(0 if ok else 1)
PY
