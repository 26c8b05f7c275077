#!/usr/bin/env bash
# The GPU evidence suites behind profiles/ and docs/BENCHMARKS.md, one gpurun call per suite:
#
#   gpurun --timeout 1100 -- 'bash tools/gpu_evidence.sh reentry'
#
# Suites:
#   reentry   GPU tests, smoke(), the default bench, a kernel + copy trace of the bench
#   pmc       rocprofv3 counter passes over a short bench (one pass per counter block budget)
#   rptests   the rocprofiler tool's GPU tests (request GPU wait under contention included)
#   config2   BASELINE config 2: Llama 7B preset, 800 ms TTFT SLO, GEMM burners, per-window attribution
#   live      config3 then config2
#   live3     the rocprof tool's GPU tests, then config3
#   live34    config3, then config4 (TP = visible GPUs)
#   headline  the headline-shape oracle test, then config4
#   branch    GPU tests, smoke, the bench with / without the span branch stream, a kernel trace
#   overhead  the shipped agent's CPU / RSS at 1M events/s (its defaults: one hardware queue)
#   config3   BASELINE config 3: rag-service + vector DB, TCP-retransmit and CPU faults, 2-fault Bayes
#   spread    the headline bench at K = 20 and K = 200, repeated on one box
#   rss       the HIP runtime's resident floor under queue / SDMA knobs
#   probe     the join's oracle GPU tests, the default bench, a kernel trace (join kernel work)
#   final     every GPU test, smoke, the bench at K = 20 and 100, a kernel + copy trace (profiles/r5_final/)
#   overhead5 the shipped agent's CPU / RSS with the shipped configuration (profiles/r5_overhead/)
#
# Every step runs under its own time limit (tools/gpu_steps.sh); a timeout or crash ends the call.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
S="bash tools/gpu_steps.sh"
B="python3 bench.py --steps 5 --warmup 2 --paced-windows 0"
P="timeout -s KILL 120 rocprofv3 --output-format csv --kernel-trace --pmc"
case "${1:-reentry}" in
  reentry)
    $S "400|gputests|python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread" \
       "200|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
       "300|bench|python -u bench.py" \
       "300|trace|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/trace -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0" ;;
  pmc)
    $S "150|pmc1|$P SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc1 -- $B" \
       "150|pmc2|$P SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc2 -- $B" \
       "150|pmc3|$P FETCH_SIZE -d gpurun_out/pmc3 -- $B" \
       "150|pmc4|$P WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc4 -- $B" ;;
  rptests)
    $S "240|rp_tests|python -u -m pytest tests/test_rocprof_tool.py -m gpu -x -v -s --timeout 150 --timeout-method thread" ;;
  config2)
    $S "600|c2_7b|python -u tools/config2_evidence.py --out gpurun_out/r4_config2_7b ${2:-}" ;;
  live2)    # the rocprof tool's GPU tests, then configs 3 and 2
    $S "300|rp_tests|python -u -m pytest tests/test_rocprof_tool.py -m gpu -x -v -s --timeout 200 --timeout-method thread" \
       "480|c3|python -u tools/config3_evidence.py --out gpurun_out/r4_config3" \
       "700|c2_7b|python -u tools/config2_evidence.py --out gpurun_out/r4_config2_7b" ;;
  live3)    # the rocprof tool's GPU tests, then config 3
    $S "300|rp_tests|python -u -m pytest tests/test_rocprof_tool.py -m gpu -x -v -s --timeout 200 --timeout-method thread" \
       "480|c3|python -u tools/config3_evidence.py --out gpurun_out/r4_config3" ;;
  live34)   # configs 3 and 4 (config 4 at TP = the box's GPU count)
    $S "480|c3|python -u tools/config3_evidence.py --out gpurun_out/r4_config3" \
       "700|c4|python -u tools/config4_evidence.py --out gpurun_out/r4_config4" ;;
  headline) # the bench-shape oracle test, then config 4 with lighter burners
    $S "400|headline|python -u -m pytest tests/test_native_engine.py -m gpu -x -v -s --timeout 360 --timeout-method thread -k headline" \
       "700|c4|python -u tools/config4_evidence.py --out gpurun_out/r4_config4 --burners-per-cpu 2 ${2:-}" ;;
  branch)   # GPU tests, then the bench with and without the span branch stream, and a kernel trace
    $S "400|gputests|python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread" \
       "200|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
       "300|bench|python -u bench.py" \
       "300|bench_nobranch|MISLO_SPAN_STREAM=0 python -u bench.py" \
       "300|bench_branch_hiprio|MISLO_SPAN_STREAM_PRIO=1 python -u bench.py" \
       "300|trace|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/trace -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0" ;;
  live)     # configs 3 and 2 back to back (the live-attribution evidence)
    $S "480|c3|python -u tools/config3_evidence.py --out gpurun_out/r4_config3" \
       "700|c2_7b|python -u tools/config2_evidence.py --out gpurun_out/r4_config2_7b" ;;
  overhead)
    $S "200|agent_oh|python -u tools/agent_overhead.py --rate 1e6 --seconds 20 --out gpurun_out/r4_agent_overhead_1Mevs.json" ;;
  config3)
    $S "480|c3|python -u tools/config3_evidence.py --out gpurun_out/r4_config3 ${2:-}" ;;
  buffers)  # windows in flight: the copy of window k waits for window k - buffers + 1's results
    for b in 3 4 5 4 3; do
      $S "200|buf_$b|python3 bench.py --steps 100 --warmup 10 --buffers $b" || exit 1
      tail -n 1 gpurun_out/buf_$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('buffers', $b, d['ms_per_step'], d['value'], d['window_copy_ms'], d['window_device_ms_compute'])"
    done ;;
  spread)  # the headline's spread on one box: K = 20 (the driver's default) and K = 200
    for i in 1 2 3; do
      $S "200|k20_$i|python3 bench.py --steps 20 --warmup 5" || exit 1
      tail -n 1 gpurun_out/k20_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('K20', d['ms_per_step'], d['value'])"
    done
    for i in 1 2; do
      $S "300|k200_$i|python3 bench.py --steps 200 --warmup 10" || exit 1
      tail -n 1 gpurun_out/k200_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('K200', d['ms_per_step'], d['value'])"
    done ;;
  final)    # round 5's final validation: every GPU test, smoke, the bench at K = 20 and 100, a kernel + copy trace
    $S "500|gputests|python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread" \
       "200|smoke|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
       "300|bench|python -u bench.py" \
       "300|bench100|python -u bench.py --steps 100 --warmup 10" \
       "300|trace|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/trace_final -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0" ;;
  overhead5) # the shipped agent at 1M events/s, shipped configuration (3 runs) and built-in defaults
    O="python -u tools/agent_overhead.py --rate 1e6 --seconds 20"
    $S "200|oh_1|$O --out gpurun_out/r5_oh_1.json" "200|oh_2|$O --out gpurun_out/r5_oh_2.json" \
       "200|oh_3|$O --out gpurun_out/r5_oh_3.json" "200|oh_bare|$O --bare --out gpurun_out/r5_oh_bare.json" ;;
  probe)    # the join's oracle tests (headline shape included), the bench, a kernel trace ($2: out tag)
    $S "420|native|python -u -m pytest tests/test_native_engine.py tests/test_gpu_engine.py -m gpu -x -v --timeout 360 --timeout-method thread" \
       "300|bench|python -u bench.py" \
       "300|trace|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_${2:-probe} -- python3 bench.py --steps 20 --warmup 3 --paced-windows 0" ;;
  rss)
    $S "120|rss_q1|GPU_MAX_HW_QUEUES=1 python tools/rss_probe.py" \
       "120|rss_q1_devq|GPU_MAX_HW_QUEUES=1 HSA_ALLOCATE_QUEUE_DEV_MEM=1 python tools/rss_probe.py" \
       "120|rss_q1_nosdma|GPU_MAX_HW_QUEUES=1 HSA_ENABLE_SDMA=0 python tools/rss_probe.py" ;;
  *) echo "unknown suite: $1" >&2; exit 2 ;;
esac
