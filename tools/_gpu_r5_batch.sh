S='bash tools/gpu_steps.sh'
$S "150|ab_r4_1|bash tools/probe_variants.sh bench r4join --steps 100 --warmup 10 --paced-windows 0" \
   "150|ab_cur_1|python -u bench.py --steps 100 --warmup 10 --paced-windows 0" \
   "150|ab_r4_2|bash tools/probe_variants.sh bench r4join --steps 100 --warmup 10 --paced-windows 0" \
   "150|ab_cur_2|python -u bench.py --steps 100 --warmup 10 --paced-windows 0" \
   "150|ab_r4_3|bash tools/probe_variants.sh bench r4join --steps 100 --warmup 10 --paced-windows 0" \
   "150|ab_cur_3|python -u bench.py --steps 100 --warmup 10 --paced-windows 0"
