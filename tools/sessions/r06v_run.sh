#!/bin/bash
# round 6: phase-A tap loads out of range instead of exec-masked (BH_DW_OOB,
# libband_hip_oob.so) against the default build, interleaved: chain / conv
# parity, the batch-32 and batch-1 mix, the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06v
mkdir -p $O
for v in oob; do
  BAND_HIP_LIB_VARIANT=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_chain_gpu.py tests/test_kernels_gpu.py > $O/${v}_tests.log 2>&1 || exit 1
  tail -1 $O/${v}_tests.log
done
for r in 1 2; do
  for v in base oob; do
    if [ $v = base ]; then unset BAND_HIP_LIB_VARIANT; else export BAND_HIP_LIB_VARIANT=$v; fi
    timeout -k 10 300 python -u tools/mix_breakdown.py --batch 32 --iters 20 --top 400 > $O/mix_b32_${v}_r$r.txt 2>&1 || exit 2
    timeout -k 10 300 python -u tools/mix_breakdown.py --batch 1 --iters 50 --top 400 > $O/mix_b1_${v}_r$r.txt 2>&1 || exit 3
  done
done
unset BAND_HIP_LIB_VARIANT
bash tools/ab_args_env.sh r06v/bench 2 "-- --no-batch1" "BAND_HIP_LIB_VARIANT=oob -- --no-batch1" || exit 4
echo done
