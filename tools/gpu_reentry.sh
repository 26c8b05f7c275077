#!/usr/bin/env bash
# Re-entry validation of HEAD: all GPU tests, smoke(), default bench, kernel trace of the bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "400|gputests|python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread" \
  "200|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|bench|python -u bench.py" \
  "300|trace|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/trace -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0"
