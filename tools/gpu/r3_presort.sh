#!/usr/bin/env bash
# span pre-sort (k_span_sort): engine GPU tests, default bench, kernel trace; posterior PMC;
# the probe's per-key-type cost split (diagnostic harness build, box copy only)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="timeout -s KILL 120 rocprofv3 --output-format csv --kernel-trace --kernel-include-regex k_posterior --pmc"
B="python3 bench.py --steps 5 --warmup 2 --paced-windows 0 --heldout 0"
tools/gpu_steps.sh \
  "300|p_tests|python -u -m pytest tests/test_native_engine.py tests/test_gpu_engine.py tests/test_agent_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread" \
  "240|p_bench|python -u bench.py" \
  "240|p_trace|rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p_trace -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0" \
  "150|p_pmc_post|$P SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD -d gpurun_out/p_pmc_post -- $B" \
  "400|pp_build|MISLO_HIP_DEFINES=-DMISLO_PROBE_PROFILE python -c 'from llm_slo_ebpf_toolkit_amd.ops import build; build.build_hip_ext(force=True, jobs=16)'" \
  "240|pp_run|python -u tools/probe_profile.py --events 2097152 --windows 4"
