set -u
for x in 0 1 2 3 4; do
  export MISLO_HIP_DEFINES="-DMISLO_EXP=$x"
  timeout -k 10 300 python -c "from llm_slo_ebpf_toolkit_amd.ops.build import build_hip_ext; build_hip_ext(force=True)" > gpurun_out/build_$x.log 2>&1 || exit 1
  timeout -k 10 120 python3 tools/stage_timing.py --wire 20 > gpurun_out/exp_$x.log 2>&1 || exit $?
  echo "exp $x $(grep -E '"join"' gpurun_out/exp_$x.log)"
done
