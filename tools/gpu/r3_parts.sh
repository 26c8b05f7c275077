#!/usr/bin/env bash
# 128 hash partitions per key type: exactness (GPU tests), throughput, kernel trace; then config 3.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "420|r3_gputests4|python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread" \
  "240|r3_bench4|python3 bench.py --steps 20 --warmup 5 --out gpurun_out/r3_bench4.json" \
  "240|r3_trace4|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_trace4 -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0 --heldout 0 --train-windows 0 --model bayes" \
  "340|r3_config3c|python -u tools/config3_evidence.py --out gpurun_out/config3c"
