#!/usr/bin/env bash
# config 2 as BASELINE names it (Llama 7B preset, TTFT SLO 800 ms, measured detection delay);
# then the probe's per-key-type cost split (diagnostic build of the kernel harness, box copy only)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "700|c2_7b|python -u tools/config2_evidence.py --out gpurun_out/r3_config2_7b" \
  "400|pp_build|MISLO_HIP_DEFINES=-DMISLO_PROBE_PROFILE python -c 'from llm_slo_ebpf_toolkit_amd.ops import build; build.build_hip_ext(force=True, jobs=16)'" \
  "240|pp_run|python -u tools/probe_profile.py --events 2097152 --windows 4"
