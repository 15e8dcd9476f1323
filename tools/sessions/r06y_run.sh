#!/bin/bash
# round 6: the latency / throughput frontier, second sweep near p99 3 ms at
# 105k (two rounds, interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06y
bash tools/ab_args_env.sh r06y/lat 2 "-- --no-batch1 --job-batch 24 --pass-target-us 400 --inflight 208" \
  "-- --no-batch1 --job-batch 24 --pass-target-us 450 --inflight 200" \
  "-- --no-batch1 --job-batch 20 --pass-target-us 500 --inflight 200" \
  "-- --no-batch1 --job-batch 24 --pass-target-us 500 --inflight 200" || exit 1
echo done
