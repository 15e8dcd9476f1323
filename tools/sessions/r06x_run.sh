#!/bin/bash
# round 6: the latency / throughput frontier on the final build - job batch
# 24, pass target 500 / 600 us, 192 / 208 / 224 requests in flight (two
# rounds, interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06x
bash tools/ab_args_env.sh r06x/lat 2 "-- --no-batch1 --job-batch 24 --pass-target-us 600 --inflight 224" \
  "-- --no-batch1 --job-batch 24 --pass-target-us 600 --inflight 192" \
  "-- --no-batch1 --job-batch 24 --pass-target-us 500 --inflight 208" \
  "-- --no-batch1 --job-batch 32 --pass-target-us 500 --inflight 224" || exit 1
echo done
