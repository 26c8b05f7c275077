#!/usr/bin/env bash
# PMC passes of the current default bench (USER24 user ring): LDS / MFMA, wave time, HBM bytes, L2.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4
B="python3 bench.py --steps 5 --warmup 2 --paced-windows 0"
P="timeout -s KILL 120 rocprofv3 --output-format csv --kernel-trace --pmc"
bash tools/gpu_steps.sh \
  "150|pmc1|$P SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc1 -- $B" \
  "150|pmc2|$P SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc2 -- $B" \
  "150|pmc3|$P FETCH_SIZE -d gpurun_out/pmc3 -- $B" \
  "150|pmc4|$P WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc4 -- $B"
