#!/bin/bash
# ring-defs: per-workgroup counter reduction, 2x grid. Oracle tests, bench, kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_engine.py tests/test_gpu_engine.py > gpurun_out/r2_tests_r.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --paced-windows 3 > gpurun_out/r2_bench_r.json 2> gpurun_out/r2_bench_r.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r2_prof8 -o run -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0 --heldout 0 > gpurun_out/r2_prof8.log 2>&1
