S='bash tools/gpu_steps.sh'
O='python -u tools/agent_overhead.py --rate 1e6 --seconds 20'
$S "420|native|python -u -m pytest tests/test_native_engine.py tests/test_gpu_engine.py -m gpu -x -v --timeout 360 --timeout-method thread" \
   "300|bench|python -u bench.py" \
   "300|trace|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_t32 -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0" \
   "200|prof|bash tools/probe_variants.sh run prof tools/probe_profile.py --windows 4" \
   "200|oh_s1|$O --out gpurun_out/r5_oh_final_1.json" \
   "200|oh_s2|$O --out gpurun_out/r5_oh_final_2.json" \
   "200|oh_s3|$O --out gpurun_out/r5_oh_final_3.json" \
   "500|gputests|python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread"
