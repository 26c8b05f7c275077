#!/usr/bin/env bash
# Round-end evidence for the current default: GPU tests, smoke, headline bench (x2), overlap
# probe, kernel/copy trace with stats, 4 PMC passes, 2-rank gloo rehearsal of the distributed
# bench on the one-GPU box. Each GPU step has its own time limit (tools/gpu_steps.sh).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4
B="python3 bench.py --steps 5 --warmup 2 --paced-windows 0"
P="timeout -s KILL 120 rocprofv3 --output-format csv --kernel-trace --pmc"
bash tools/gpu_steps.sh \
  "300|gputests|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "150|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "200|bench|python3 bench.py --steps 200 --warmup 10" \
  "200|bench2|python3 bench.py --steps 200 --warmup 10" \
  "150|overlap|python3 tools/overlap_probe.py" \
  "240|stats|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof -- python3 bench.py --steps 10 --warmup 3 --paced-windows 0" \
  "150|pmc1|$P SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc1 -- $B" \
  "150|pmc2|$P SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc2 -- $B" \
  "150|pmc3|$P FETCH_SIZE -d gpurun_out/pmc3 -- $B" \
  "150|pmc4|$P WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc4 -- $B" \
  "300|gloo2|MISLO_BENCH_GPU_OF_RANK=0 MISLO_DIST_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --paced-windows 1"
