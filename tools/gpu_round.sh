#!/usr/bin/env bash
# One validation + profiling pass on the GPU box: GPU tests, smoke(), the headline bench, a
# rocprofv3 kernel/copy trace of the bench, and rocprofv3 PMC passes (one counter group per run,
# each within the per-block limits) for tools/pmc_summary.py. Every GPU step has its own time
# limit; a timeout / crash (rc >= 124) ends the script (tools/gpu_steps.sh).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 5 --warmup 2 --paced-windows 0"
P="timeout -s KILL 120 rocprofv3 --output-format csv --kernel-trace --pmc"
exec_steps=(
  "300|gputests|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread"
  "200|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'"
  "240|bench|python3 bench.py --steps 100 --warmup 10"
  "240|stats|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof -- python3 bench.py --steps 10 --warmup 3 --paced-windows 0"
  "150|pmc1|$P SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc1 -- $B"
  "150|pmc2|$P SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc2 -- $B"
  "150|pmc3|$P FETCH_SIZE -d gpurun_out/pmc3 -- $B"
  "150|pmc4|$P WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc4 -- $B"
)
bash tools/gpu_steps.sh "${exec_steps[@]}"
