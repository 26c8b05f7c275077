#!/usr/bin/env bash
# USER24 user-space records: GPU tests, smoke, bench A/B against USER32 on the same box.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "420|gputests|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "150|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "200|bench24|python3 bench.py --steps 100 --warmup 10" \
  "200|bench32|python3 bench.py --steps 100 --warmup 10 --user-rec 32" \
  "200|bench24b|python3 bench.py --steps 100 --warmup 10" \
  "240|stats24|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof24 -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0"
