#!/bin/bash
# round 6: fewer GPU workers per GPU on the final build (6 / 7, in flight
# scaled; 6 with job batch 40), interleaved against the default 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06ab
bash tools/ab_args_env.sh r06ab/w 2 "-- --no-batch1" \
  "-- --no-batch1 --workers-per-gpu 6 --inflight 240" \
  "-- --no-batch1 --workers-per-gpu 7 --inflight 280" \
  "-- --no-batch1 --workers-per-gpu 6 --job-batch 40 --inflight 300" || exit 1
echo done
