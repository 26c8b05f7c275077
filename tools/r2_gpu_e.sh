#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --paced-windows 0 > gpurun_out/r2_bench11_s2.json 2> gpurun_out/r2_bench11_s2.err &&
MISLO_COPY_STREAMS=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --paced-windows 0 > gpurun_out/r2_bench11_s1.json 2> gpurun_out/r2_bench11_s1.err &&
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --paced-windows 0 > gpurun_out/r2_bench11_s2b.json 2> gpurun_out/r2_bench11_s2b.err
