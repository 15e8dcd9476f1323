#!/bin/bash
# round 6: ROCr / HIP runtime knobs against the default bench line (a host
# thread of the HIP runtime runs near one full core in every headline run):
# polled signal waits (HSA_ENABLE_INTERRUPT=0), blit-kernel copies instead
# of SDMA (HSA_ENABLE_SDMA=0), kernel arguments in device memory
# (HIP_FORCE_DEV_KERNARG=1); interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06ad
bash tools/ab_args_env.sh r06ad/rt 2 "-- --no-batch1" "HSA_ENABLE_INTERRUPT=0 -- --no-batch1" \
  "HSA_ENABLE_SDMA=0 -- --no-batch1" "HIP_FORCE_DEV_KERNARG=1 -- --no-batch1" || exit 1
echo done
