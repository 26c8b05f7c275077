#!/usr/bin/env bash
# posterior model in LDS, fused window head: engine GPU tests, default bench, kernel trace;
# HIP host-memory floor on the null stream (one queue?)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "300|f_tests|python -u -m pytest tests/test_native_engine.py tests/test_gpu_engine.py tests/test_agent_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread" \
  "240|f_bench|python -u bench.py" \
  "240|f_trace|rocprofv3 --kernel-trace --output-format csv -d gpurun_out/f_trace -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0" \
  "60|f_rss_null|GPU_MAX_HW_QUEUES=1 build/hip_rss_floor null"
