#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_engine.py tests/test_agent_gpu.py > gpurun_out/r2_tests_f.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 > gpurun_out/r2_bench9.json 2> gpurun_out/r2_bench9.err
