#!/usr/bin/env bash
# One GPU-box validation pass: GPU tests, smoke(), per-stage timing (wire 20 / 32) and the
# headline bench. Each step has its own time limit; a timeout / crash ends the script.
set -u
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/gputests.log 2>&1; rc=$?; tail -15 gpurun_out/gputests.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
for w in 16 20 32; do timeout -k 10 120 python3 tools/stage_timing.py --wire $w > gpurun_out/st_$w.log 2>&1 || exit $?; echo "wire $w $(grep -E '"(decode|join|h2d|total_ms)"' gpurun_out/st_$w.log | tr -d '\n')"; done
timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --wire ${BENCH_WIRE:-20} > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_issue_us_per_window'], d['macro_f1'], d['agent_cpu_overhead_pct'], d['host_encode_ms_per_window'])"
timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --wire 16 > gpurun_out/bench16.log 2>&1 || exit $?
tail -1 gpurun_out/bench16.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('wire16', d['value'], d['ms_per_step'], d['host_encode_ms_per_window'])"
