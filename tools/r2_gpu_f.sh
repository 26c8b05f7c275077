#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/config2
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_rocprof_tool.py > gpurun_out/r2_rocprof_test.log 2>&1 &&
timeout -k 10 600 python -u tools/config2_evidence.py --out gpurun_out/config2 > gpurun_out/config2/stdout.log 2>&1
