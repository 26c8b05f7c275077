#!/usr/bin/env bash
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "300|r3_tooltests2|python -u -m pytest tests/test_rocprof_tool.py -m gpu -x -v --timeout 200 --timeout-method thread" \
  "340|r3_config3d|python -u tools/config3_evidence.py --out gpurun_out/config3d" \
  "120|rss_q1|GPU_MAX_HW_QUEUES=1 python tools/rss_probe.py" \
  "120|rss_q1_devq|GPU_MAX_HW_QUEUES=1 HSA_ALLOCATE_QUEUE_DEV_MEM=1 python tools/rss_probe.py" \
  "120|rss_q1_maxq1|GPU_MAX_HW_QUEUES=1 HSA_MAX_QUEUES=1 python tools/rss_probe.py" \
  "120|rss_q1_nosdma|GPU_MAX_HW_QUEUES=1 HSA_ENABLE_SDMA=0 python tools/rss_probe.py"
