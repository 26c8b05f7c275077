#!/usr/bin/env bash
# Kernel trace (per-window phases, halo on) + 4 PMC passes of the agent-default bench, then the
# config-3 evidence run again (rocprof queue delay from the enqueue's return, per-process
# run-queue delay).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 5 --warmup 2 --paced-windows 0 --heldout 0 --train-windows 0 --model bayes"
P="timeout -s KILL 120 rocprofv3 --output-format csv --kernel-trace --pmc"
bash tools/gpu_steps.sh \
  "240|r3_trace|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_trace -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0 --heldout 0 --train-windows 0 --model bayes" \
  "150|r3_pmc1|$P SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/r3_pmc1 -- $B" \
  "150|r3_pmc2|$P SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/r3_pmc2 -- $B" \
  "150|r3_pmc3|$P FETCH_SIZE -d gpurun_out/r3_pmc3 -- $B" \
  "150|r3_pmc4|$P WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/r3_pmc4 -- $B" \
  "340|r3_config3b|python -u tools/config3_evidence.py --out gpurun_out/config3b"
