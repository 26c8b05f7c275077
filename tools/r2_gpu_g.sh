#!/bin/bash
# USER32 user-space records: GPU oracle tests (both record sizes), the rocprof tool writing
# either size, the bench at 32 and 64 bytes, and the device-memory RSS probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_engine.py tests/test_gpu_engine.py tests/test_agent_gpu.py > gpurun_out/r2_tests_g.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_rocprof_tool.py > gpurun_out/r2_rocprof_g.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 --user-rec 32 > gpurun_out/r2_bench_u32.json 2> gpurun_out/r2_bench_u32.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 --user-rec 64 > gpurun_out/r2_bench_u64.json 2> gpurun_out/r2_bench_u64.err &&
timeout -k 10 120 python -u tools/vram_rss_probe.py > gpurun_out/r2_vram_rss.log 2>&1
