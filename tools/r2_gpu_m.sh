#!/bin/bash
# head load on the compute stream: tests, bench, copy/kernel timeline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_engine.py tests/test_gpu_engine.py tests/test_agent_gpu.py > gpurun_out/r2_tests_m.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 > gpurun_out/r2_bench_m.json 2> gpurun_out/r2_bench_m.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 > gpurun_out/r2_bench_m2.json 2> gpurun_out/r2_bench_m2.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r2_prof6 -o run -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0 > gpurun_out/r2_prof6.log 2>&1
