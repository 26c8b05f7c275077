S='bash tools/gpu_steps.sh'
$S "500|gputests|python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread" \
   "200|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
   "300|bench|python -u bench.py" \
   "300|bench100|python -u bench.py --steps 100 --warmup 10" \
   "300|bench100b|python -u bench.py --steps 100 --warmup 10" \
   "300|trace|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/trace_final3 -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0"
