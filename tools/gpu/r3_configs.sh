#!/usr/bin/env bash
# rocprof tool tests (queue predecessors from the enqueue order); config 2 as BASELINE names it (Llama 7B preset, TTFT SLO 800 ms, measured detection delay);
# config 3 with a harder CPU fault (12 burners per victim CPU); the shipped agent's overhead at 1M events/s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "200|rp_tests|python -u -m pytest tests/test_rocprof_tool.py -m gpu -x -v --timeout 150 --timeout-method thread" \
  "480|c2_7b|python -u tools/config2_evidence.py --out gpurun_out/r3_config2_7b" \
  "420|c3_b12|python -u tools/config3_evidence.py --out gpurun_out/r3_config3_b12 --burners-per-cpu 12 --procfs-ms 25" \
  "200|agent_oh|python -u tools/agent_overhead.py --rate 1e6 --seconds 20 --out gpurun_out/r3_agent_overhead_1Mevs.json"
