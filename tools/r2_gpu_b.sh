#!/bin/bash
# agent exit check: stack dump (SIGUSR1) if it hangs, then the agent GPU test
set -o pipefail
mkdir -p gpurun_out
timeout -s USR1 -k 15 60 python -u -m llm_slo_ebpf_toolkit_amd.cli.agent --engine gpu --source replay --count 4 --window-ms 500 --window-events 262144 --window-spans 4096 --window-groups 64 --output jsonl --output-path gpurun_out/r2_agent_attr3.jsonl --metrics-bind "" --scenario full > gpurun_out/r2_agent3.log 2>&1
echo "agent rc=$?" >> gpurun_out/r2_agent3.log
timeout -k 10 150 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_agent_gpu.py > gpurun_out/r2_agent_test.log 2>&1
