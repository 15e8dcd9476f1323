#!/bin/bash
# round 6: MFMA accumulators in VGPRs (-mllvm -amdgpu-mfma-vgpr-form, no
# AGPR copies; libband_hip_vgpr.so) against the default build - chain and
# conv parity on the variant, then the batch-32 / batch-1 mix and the
# default bench line, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06q
mkdir -p $O
BAND_HIP_LIB_VARIANT=vgpr timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_chain_gpu.py tests/test_kernels_gpu.py > $O/vgpr_tests.log 2>&1 || exit 1
tail -1 $O/vgpr_tests.log
for r in 1 2; do
  for v in base vgpr; do
    if [ $v = vgpr ]; then export BAND_HIP_LIB_VARIANT=vgpr; else unset BAND_HIP_LIB_VARIANT; fi
    timeout -k 10 300 python -u tools/mix_breakdown.py --batch 32 --iters 20 --top 400 > $O/mix_b32_${v}_r$r.txt 2>&1 || exit 2
    timeout -k 10 300 python -u tools/mix_breakdown.py --batch 1 --iters 50 --top 400 > $O/mix_b1_${v}_r$r.txt 2>&1 || exit 3
  done
done
unset BAND_HIP_LIB_VARIANT
bash tools/ab_args_env.sh r06q/bench 2 "-- --no-batch1" "BAND_HIP_LIB_VARIANT=vgpr -- --no-batch1" || exit 4
echo done
