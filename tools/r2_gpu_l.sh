#!/bin/bash
# USER32 agent rings + smaller replay rings, queue-delay threshold 2 ms: tests, bench (default and
# 2 hardware queues), agent overhead (default and 2 hardware queues), config-2.
set -o pipefail
mkdir -p gpurun_out/config2e
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_engine.py tests/test_gpu_engine.py tests/test_agent_gpu.py > gpurun_out/r2_tests_l.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 > gpurun_out/r2_bench_l.json 2> gpurun_out/r2_bench_l.err &&
GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 > gpurun_out/r2_bench_l_q2.json 2> gpurun_out/r2_bench_l_q2.err &&
timeout -k 10 200 python -u tools/agent_overhead.py --rate 1e6 --seconds 12 --out gpurun_out/r2_agent_overhead4.json > gpurun_out/r2_agent_overhead4.log 2>&1 &&
GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python -u tools/agent_overhead.py --rate 1e6 --seconds 12 --out gpurun_out/r2_agent_overhead4_q2.json > gpurun_out/r2_agent_overhead4_q2.log 2>&1 &&
timeout -k 10 600 python -u tools/config2_evidence.py --out gpurun_out/config2e > gpurun_out/config2e/stdout.log 2>&1
