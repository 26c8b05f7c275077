#!/bin/bash
# native engine after the trace-id table / imports refactor: GPU tests, smoke, bench (halo off / on)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_engine.py tests/test_gpu_engine.py tests/test_agent_gpu.py > gpurun_out/r2_tests_e.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench5.json 2> gpurun_out/r2_bench5.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --halo-ms 2000 > gpurun_out/r2_bench5_halo.json 2> gpurun_out/r2_bench5_halo.err
