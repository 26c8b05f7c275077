#!/usr/bin/env bash
# Run-to-run spread of the default bench (the driver's K) on one box.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "200|rep1|python3 bench.py" \
  "200|rep2|python3 bench.py" \
  "200|rep3|python3 bench.py" \
  "200|rep4|python3 bench.py --steps 200 --warmup 10"
