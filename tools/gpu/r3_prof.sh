#!/usr/bin/env bash
# Kernel trace (per-window phases, halo on) + 4 PMC passes of the agent-default bench, and the
# default bench for the quality numbers.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 5 --warmup 2 --paced-windows 0 --heldout 0 --train-windows 0 --model bayes"
P="timeout -s KILL 120 rocprofv3 --output-format csv --kernel-trace --pmc"
bash tools/gpu_steps.sh \
  "420|r3_gputests2|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "200|r3_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r3_bench2|python3 bench.py --steps 20 --warmup 5 --out gpurun_out/r3_bench2.json" \
  "240|r3_trace|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_trace -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0 --heldout 0 --train-windows 0 --model bayes" \
  "150|r3_pmc1|$P SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/r3_pmc1 -- $B" \
  "150|r3_pmc2|$P SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/r3_pmc2 -- $B" \
  "150|r3_pmc3|$P FETCH_SIZE -d gpurun_out/r3_pmc3 -- $B" \
  "150|r3_pmc4|$P WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/r3_pmc4 -- $B" \
"120|rss_q1|GPU_MAX_HW_QUEUES=1 python tools/rss_probe.py" \
  "120|rss_q1_devq|GPU_MAX_HW_QUEUES=1 HSA_ALLOCATE_QUEUE_DEV_MEM=1 python tools/rss_probe.py" \
  "120|rss_q1_nosdma|GPU_MAX_HW_QUEUES=1 HSA_ENABLE_SDMA=0 python tools/rss_probe.py" \
  "120|rss_q1_devq_nosdma|GPU_MAX_HW_QUEUES=1 HSA_ALLOCATE_QUEUE_DEV_MEM=1 HSA_ENABLE_SDMA=0 python tools/rss_probe.py" \
  "120|rss_q2_devq|GPU_MAX_HW_QUEUES=2 HSA_ALLOCATE_QUEUE_DEV_MEM=1 python tools/rss_probe.py"
