#!/usr/bin/env bash
# Config-2 evidence with the agent's default USER24 ring: Llama on the GPU with the rocprof tool,
# the agent's GPU engine on its rings, injected GPU contention.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/config2_user24
timeout -k 10 600 python -u tools/config2_evidence.py --out gpurun_out/config2_user24 > gpurun_out/config2_user24/stdout.log 2>&1
