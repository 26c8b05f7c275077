#!/usr/bin/env bash
# GPU tests + smoke, headline bench twice, overlap probe, kernel stats profile.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
bash tools/gpu_steps.sh \
  "300|gputests|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "150|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "200|bench|python3 bench.py --steps 200 --warmup 10" \
  "200|bench2|python3 bench.py --steps 200 --warmup 10" \
  "150|overlap|python3 tools/overlap_probe.py" \
  "240|stats|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof -- python3 bench.py --steps 10 --warmup 3 --paced-windows 0"
