#!/usr/bin/env bash
# GPU tests, then the headline bench with the 20-byte (EVENT20T) and 24-byte (EVENT24) probe
# ring records back to back on the same box.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
tail -3 gpurun_out/gputests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
for w in ${WIRES:-20t 16t 20t 16t}; do
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 10 --wire $w > gpurun_out/bench_$w.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('wire', '$w', d['ms_per_step'], d['value'], d['macro_f1'], d['agent_cpu_overhead_pct'])"
done
timeout -k 10 120 python3 tools/overlap_probe.py --wire 21 > gpurun_out/overlap.log 2>&1 && tail -1 gpurun_out/overlap.log
