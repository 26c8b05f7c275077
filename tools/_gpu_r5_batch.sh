S='bash tools/gpu_steps.sh'
$S "150|sw_g512|MISLO_PROBE_GRID=512 python -u bench.py --steps 100 --warmup 10 --paced-windows 0" \
   "150|sw_g768b|MISLO_PROBE_GRID=768 python -u bench.py --steps 100 --warmup 10 --paced-windows 0" \
   "150|sw_base3|python -u bench.py --steps 100 --warmup 10 --paced-windows 0" \
   "150|sw_g640|MISLO_PROBE_GRID=640 python -u bench.py --steps 100 --warmup 10 --paced-windows 0" \
   "150|sw_g768c|MISLO_PROBE_GRID=768 python -u bench.py --steps 100 --warmup 10 --paced-windows 0" \
   "150|sw_base4|python -u bench.py --steps 100 --warmup 10 --paced-windows 0"
