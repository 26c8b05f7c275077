#!/usr/bin/env bash
# GPU tests (2-fault device refit), smoke, the default bench, then the config-3 evidence run.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "400|r3_gputests3|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "180|r3_smoke3|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "240|r3_bench3|python3 bench.py --steps 20 --warmup 5 --out gpurun_out/r3_bench3.json" \
  "340|r3_config3|python -u tools/config3_evidence.py --out gpurun_out/config3"
