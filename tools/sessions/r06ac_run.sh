#!/bin/bash
# round 6: the tuner's isolated choices under concurrency - the default bench
# line against the same run without the stage chain forms and without the
# tile chain forms (BAND_HIP_FUSION=nostage / notile), interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06ac
bash tools/ab_args_env.sh r06ac/f 3 "-- --no-batch1" "BAND_HIP_FUSION=nostage -- --no-batch1" \
  "BAND_HIP_FUSION=notile -- --no-batch1" || exit 1
echo done
