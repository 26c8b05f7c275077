#!/bin/bash
# round-2 evidence batch: bench (1 GPU), rocprof of the native engine, agent replay exit check
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench4.json 2> gpurun_out/r2_bench4.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r2_prof4 -o run -- python tools/profile_engine.py --windows 12 > gpurun_out/r2_prof4.log 2>&1 &&
timeout -k 10 240 python -u -m llm_slo_ebpf_toolkit_amd.cli.agent --engine gpu --source replay --count 4 --window-ms 500 --window-events 262144 --window-spans 4096 --window-groups 64 --output jsonl --output-path gpurun_out/r2_agent_attr2.jsonl --metrics-bind "" --scenario full > gpurun_out/r2_agent2.log 2>&1
