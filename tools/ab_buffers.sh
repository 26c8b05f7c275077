set -u
for b in 2 3 2 3; do
  timeout -k 10 120 python3 tools/overlap_probe.py --buffers $b > gpurun_out/ov_$b.log 2>&1 || exit 1; tail -1 gpurun_out/ov_$b.log
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 10 --paced-windows 0 --buffers $b > gpurun_out/b_$b.log 2>&1 || exit 1
  tail -1 gpurun_out/b_$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench buffers', $b, d['ms_per_step'], d['value'])"
done
