#!/usr/bin/env bash
# Where the agent's resident memory goes, under runtime knobs that may move the per-queue
# context-save areas (CWSR) or the queues themselves out of host memory.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "120|rss_q1|GPU_MAX_HW_QUEUES=1 python tools/rss_probe.py" \
  "120|rss_q1_devq|GPU_MAX_HW_QUEUES=1 HSA_ALLOCATE_QUEUE_DEV_MEM=1 python tools/rss_probe.py" \
  "120|rss_q1_nosdma|GPU_MAX_HW_QUEUES=1 HSA_ENABLE_SDMA=0 python tools/rss_probe.py" \
  "120|rss_q1_devq_nosdma|GPU_MAX_HW_QUEUES=1 HSA_ALLOCATE_QUEUE_DEV_MEM=1 HSA_ENABLE_SDMA=0 python tools/rss_probe.py" \
  "120|rss_q2_devq|GPU_MAX_HW_QUEUES=2 HSA_ALLOCATE_QUEUE_DEV_MEM=1 python tools/rss_probe.py" \
  "120|rss_q1_maxq1|GPU_MAX_HW_QUEUES=1 HSA_MAX_QUEUES=1 python tools/rss_probe.py"
