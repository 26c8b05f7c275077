#!/bin/bash
# single-GPU engine without a comm stream: tests, bench, RSS (default / 2 hardware queues),
# agent overhead, config-2 with the GPU signal histograms.
set -o pipefail
mkdir -p gpurun_out/config2d
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_engine.py tests/test_gpu_engine.py tests/test_agent_gpu.py > gpurun_out/r2_tests_k.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 > gpurun_out/r2_bench_k.json 2> gpurun_out/r2_bench_k.err &&
timeout -k 10 120 python -u tools/rss_probe.py > gpurun_out/r2_rss_probe3.log 2>&1 &&
GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python -u tools/rss_probe.py > gpurun_out/r2_rss_probe3_q2.log 2>&1 &&
timeout -k 10 200 python -u tools/agent_overhead.py --rate 1e6 --seconds 12 --out gpurun_out/r2_agent_overhead3.json > gpurun_out/r2_agent_overhead3.log 2>&1 &&
timeout -k 10 600 python -u tools/config2_evidence.py --out gpurun_out/config2d > gpurun_out/config2d/stdout.log 2>&1
