#!/bin/bash
# GPU tests (USER32 variants included), rocprof tool at both record sizes, bench at 32/64-byte
# user records, a kernel profile of the engine, the device-memory RSS probe, then the config-2
# evidence run.
set -o pipefail
mkdir -p gpurun_out/config2
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_engine.py tests/test_gpu_engine.py tests/test_agent_gpu.py > gpurun_out/r2_tests_g.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 --user-rec 32 > gpurun_out/r2_bench_u32.json 2> gpurun_out/r2_bench_u32.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --paced-windows 0 --user-rec 64 > gpurun_out/r2_bench_u64.json 2> gpurun_out/r2_bench_u64.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r2_prof5 -o run -- python tools/profile_engine.py --windows 12 > gpurun_out/r2_prof5.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_rocprof_tool.py > gpurun_out/r2_rocprof_g.log 2>&1 &&
timeout -k 10 120 python -u tools/vram_rss_probe.py > gpurun_out/r2_vram_rss.log 2>&1 &&
timeout -k 10 600 python -u tools/config2_evidence.py --out gpurun_out/config2 > gpurun_out/config2/stdout.log 2>&1
