S='bash tools/gpu_steps.sh'
$S "560|c3|python -u tools/config3_evidence.py --out gpurun_out/r5_config3_retrieval"
