#!/usr/bin/env bash
# resident-generation halo: engine GPU tests, default bench, kernel trace of the agent-default bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "400|g_tests|python -u -m pytest tests/test_native_engine.py tests/test_gpu_engine.py -m gpu -x -v --timeout 150 --timeout-method thread" \
  "300|g_bench|python -u bench.py" \
  "300|g_trace|rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g_trace -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0 --heldout 0 --train-windows 0 --model bayes"
