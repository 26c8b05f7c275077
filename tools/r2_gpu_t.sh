#!/bin/bash
# agent RSS with one hardware queue
set -o pipefail
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=1 timeout -k 10 200 python -u tools/agent_overhead.py --rate 1e6 --seconds 10 --out gpurun_out/r2_agent_overhead5_q1.json > gpurun_out/r2_agent_overhead5_q1.log 2>&1 &&
GPU_MAX_HW_QUEUES=1 timeout -k 10 120 python -u tools/rss_probe.py > gpurun_out/r2_rss_probe_q1.log 2>&1
