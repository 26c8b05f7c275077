#!/bin/bash
# request trace tagging (rocprof tool) test, engine RSS breakdown, config-2 with request-tagged
# GPU records, halo and the GPU-aware expert model.
set -o pipefail
mkdir -p gpurun_out/config2c
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_rocprof_tool.py > gpurun_out/r2_rocprof_j.log 2>&1 &&
timeout -k 10 120 python -u tools/rss_probe.py > gpurun_out/r2_rss_probe2.log 2>&1 &&
timeout -k 10 600 python -u tools/config2_evidence.py --out gpurun_out/config2c > gpurun_out/config2c/stdout.log 2>&1
