#!/bin/bash
# round 6: the latency point on the final kernels (MFMA stem, multi-row
# resize): job batch x pass target x in flight near p99 3 ms at 105k,
# two rounds interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06al
bash tools/ab_args_env.sh r06al/lat 2 "-- --no-batch1 --job-batch 24 --pass-target-us 500 --inflight 200" \
  "-- --no-batch1 --job-batch 24 --pass-target-us 450 --inflight 200" \
  "-- --no-batch1 --job-batch 24 --pass-target-us 450 --inflight 208" \
  "-- --no-batch1 --job-batch 24 --pass-target-us 400 --inflight 200" || exit 1
echo done
