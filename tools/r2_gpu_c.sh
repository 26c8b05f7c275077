#!/bin/bash
# agent GPU tests (run loop, rag-service e2e) and the agent's own CPU / RSS overhead at 1M ev/s
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_agent_gpu.py > gpurun_out/r2_agent_test2.log 2>&1 &&
timeout -k 10 240 python -u tools/agent_overhead.py --rate 1e6 --seconds 20 --out gpurun_out/r2_agent_overhead.json > gpurun_out/r2_agent_overhead.log 2>&1
