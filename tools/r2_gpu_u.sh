#!/usr/bin/env bash
# Re-entry validation of the committed tree: GPU tests, smoke, headline bench.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "400|gputests|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "150|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "200|bench|python3 bench.py" \
  "180|rccl_pair|python3 -u tools/rccl_pair_probe.py"
