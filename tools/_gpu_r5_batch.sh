S='bash tools/gpu_steps.sh'
$S "420|native|python -u -m pytest tests/test_native_engine.py tests/test_gpu_engine.py tests/test_rccl_single.py -m gpu -x -v --timeout 360 --timeout-method thread" \
   "150|ab_prev_1|bash tools/probe_variants.sh bench prev --steps 100 --warmup 10 --paced-windows 0" \
   "150|ab_cur_1|python -u bench.py --steps 100 --warmup 10 --paced-windows 0" \
   "150|ab_prev_2|bash tools/probe_variants.sh bench prev --steps 100 --warmup 10 --paced-windows 0" \
   "150|ab_cur_2|python -u bench.py --steps 100 --warmup 10 --paced-windows 0" \
   "150|ab_prev_3|bash tools/probe_variants.sh bench prev --steps 100 --warmup 10 --paced-windows 0" \
   "150|ab_cur_3|python -u bench.py --steps 100 --warmup 10 --paced-windows 0" \
   "300|trace|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_merged -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0"
