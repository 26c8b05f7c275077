#!/usr/bin/env bash
# Round-3 GPU check: GPU tests, the headline bench (training + halo, agent defaults), a 1-HW-queue bench.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "420|r3_gputests|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "300|r3_bench|python3 bench.py --steps 20 --warmup 5 --out gpurun_out/r3_bench.json --export-model gpurun_out/r3_model.safetensors" \
  "300|r3_bench_q1|python3 bench.py --steps 20 --warmup 5 --hw-queues 1 --out gpurun_out/r3_bench_q1.json"
