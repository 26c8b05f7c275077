#!/usr/bin/env bash
# USER24 default: full GPU tests, smoke, headline bench (x2).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "420|gputests|python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread" \
  "150|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "200|bench|python3 bench.py" \
  "200|bench_k100|python3 bench.py --steps 100 --warmup 10"
