#!/bin/bash
# default bench (as the driver runs it), then 4 PMC passes over a short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r2_bench_default.json 2> gpurun_out/r2_bench_default.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
B="python3 bench.py --steps 5 --warmup 2 --paced-windows 0 --heldout 0" &&
P="timeout -s KILL 150 rocprofv3 --output-format csv --kernel-trace --pmc" &&
$P SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/r2_pmc1 -- $B > gpurun_out/r2_pmc1.log 2>&1 &&
$P SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/r2_pmc2 -- $B > gpurun_out/r2_pmc2.log 2>&1 &&
$P FETCH_SIZE -d gpurun_out/r2_pmc3 -- $B > gpurun_out/r2_pmc3.log 2>&1 &&
$P WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/r2_pmc4 -- $B > gpurun_out/r2_pmc4.log 2>&1
