#!/bin/bash
# bench at several K with rings sized for the whole run
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 > gpurun_out/r2_bench_s100.json 2> gpurun_out/r2_bench_s100.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench_s20.json 2> gpurun_out/r2_bench_s20.err &&
timeout -k 10 300 python -u bench.py > gpurun_out/r2_bench_sdef.json 2> gpurun_out/r2_bench_sdef.err
