#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 > gpurun_out/r2_b15.json 2> gpurun_out/r2_b15.err &&
MISLO_SPIN_WAIT=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 --buffers 4 > gpurun_out/r2_b15_s4.json 2> gpurun_out/r2_b15_s4.err
