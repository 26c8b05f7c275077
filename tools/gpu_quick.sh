#!/usr/bin/env bash
# Quick GPU check after a kernel change: GPU tests, headline bench, kernel stats profile.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "300|gputests|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "240|bench|python3 bench.py --steps 100 --warmup 10" \
  "240|stats|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof -- python3 bench.py --steps 10 --warmup 3 --paced-windows 0" \
  "${@}"
