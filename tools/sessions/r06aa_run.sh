#!/bin/bash
# round 6: concurrency knobs on the final build - 8 hardware queues, 10 / 12
# GPU workers per GPU (in flight scaled with them), interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06aa
bash tools/ab_args_env.sh r06aa/conc 2 "-- --no-batch1 --latency-point ''" \
  "GPU_MAX_HW_QUEUES=8 -- --no-batch1 --latency-point ''" \
  "-- --no-batch1 --latency-point '' --workers-per-gpu 10 --inflight 400" \
  "-- --no-batch1 --latency-point '' --workers-per-gpu 12 --inflight 480" || exit 1
echo done
