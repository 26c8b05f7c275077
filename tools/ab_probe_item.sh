set -u
for it in ${ITEMS:-2048 4096 8192 2048 4096 8192}; do
  MISLO_PROBE_ITEM=$it timeout -k 10 200 python3 bench.py --steps 200 --warmup 10 --paced-windows 0 > gpurun_out/bi_$it.log 2>&1 || exit 1
  tail -1 gpurun_out/bi_$it.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('item', $it, d['ms_per_step'], d['value'])"
  MISLO_PROBE_ITEM=$it timeout -k 10 100 python3 tools/overlap_probe.py > gpurun_out/oi_$it.log 2>&1 || exit 1; tail -1 gpurun_out/oi_$it.log
done
