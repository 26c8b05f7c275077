#!/usr/bin/env bash
# wave-level span sort, posterior over 4 waves per row group: all GPU tests, smoke, default bench,
# kernel trace of the default bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "400|w_tests|python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread" \
  "200|w_smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "240|w_bench|python -u bench.py" \
  "240|w_trace|rocprofv3 --kernel-trace --output-format csv -d gpurun_out/w_trace -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0"
