#!/usr/bin/env bash
# The shipped agent at 1M events/s with the USER24 user ring (its default now): CPU, RSS. The box
# exports GPU_MAX_HW_QUEUES=4, which wins over the agent's default of one queue: set it to 1 here.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "200|agent_overhead24|GPU_MAX_HW_QUEUES=1 python -u tools/agent_overhead.py --rate 1e6 --seconds 10 --out gpurun_out/r2_agent_overhead_user24.json"
