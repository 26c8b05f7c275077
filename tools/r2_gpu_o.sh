#!/bin/bash
# the driver's round-end GPU tiers: the whole gpu-marked suite, then smoke().
set -o pipefail
mkdir -p gpurun_out
df -h /dev/shm > gpurun_out/r2_shm.txt 2>&1
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 250 --timeout-method thread > gpurun_out/r2_gpu_all.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke3.log 2>&1
