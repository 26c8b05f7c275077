S='bash tools/gpu_steps.sh'
$S "560|c3|python -u tools/config3_evidence.py --out gpurun_out/r5f_config3" \
   "560|c4|python -u tools/config4_evidence.py --out gpurun_out/r5f_config4"
