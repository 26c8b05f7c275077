#!/usr/bin/env bash
# probe prefetch depth 2: exactness, throughput, kernel trace, PMC of the probe; config 3.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 5 --warmup 2 --paced-windows 0 --heldout 0 --train-windows 0 --model bayes"
P="timeout -s KILL 120 rocprofv3 --output-format csv --kernel-trace --pmc"
bash tools/gpu_steps.sh \
  "420|r3_gputests5|python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread" \
  "240|r3_bench5|python3 bench.py --steps 20 --warmup 5 --out gpurun_out/r3_bench5.json" \
  "240|r3_trace5|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_trace5 -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0 --heldout 0 --train-windows 0 --model bayes" \
  "150|r3_pmc5a|$P SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/r3_pmc5a -- $B" \
  "150|r3_pmc5b|$P FETCH_SIZE -d gpurun_out/r3_pmc5b -- $B" \
  "340|r3_config3c|python -u tools/config3_evidence.py --out gpurun_out/config3c"
