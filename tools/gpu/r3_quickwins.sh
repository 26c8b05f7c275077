#!/usr/bin/env bash
# decode scalar atomics per workgroup, posterior pair masks in LDS: engine GPU tests, default
# bench, kernel trace of the default bench; HIP runtime host-memory floor (native probe)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "300|q_tests|python -u -m pytest tests/test_native_engine.py tests/test_gpu_engine.py -m gpu -x -v --timeout 150 --timeout-method thread" \
  "240|q_bench|python -u bench.py" \
  "240|q_trace|rocprofv3 --kernel-trace --output-format csv -d gpurun_out/q_trace -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0" \
  "60|q_rss|GPU_MAX_HW_QUEUES=1 build/hip_rss_floor" \
  "60|q_rss4|build/hip_rss_floor"
