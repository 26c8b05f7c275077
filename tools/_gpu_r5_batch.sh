S='bash tools/gpu_steps.sh'
$S "420|native|python -u -m pytest tests/test_native_engine.py tests/test_gpu_engine.py -m gpu -x -v --timeout 360 --timeout-method thread" \
   "300|bench|python -u bench.py" \
   "300|bench100|python -u bench.py --steps 100 --warmup 10" \
   "300|trace|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_wave -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0" \
   "200|prof|bash tools/probe_variants.sh run prof tools/probe_profile.py --windows 4"
