#!/bin/bash
# RSS probe (device allocations), GPU tests incl. the agent, bench with the held-out scenario
# set, config-2 evidence with the GPU-aware expert model.
set -o pipefail
mkdir -p gpurun_out/config2b
timeout -k 10 120 python -u tools/vram_rss_probe.py > gpurun_out/r2_vram_rss2.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_engine.py tests/test_gpu_engine.py tests/test_agent_gpu.py > gpurun_out/r2_tests_i.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 > gpurun_out/r2_bench_i.json 2> gpurun_out/r2_bench_i.err &&
timeout -k 10 600 python -u tools/config2_evidence.py --out gpurun_out/config2b > gpurun_out/config2b/stdout.log 2>&1
