#!/bin/bash
# round 5: depthwise channel groups per wave per round in the chain kernel's
# DA = 2 forms (BH_CHAIN_PA 2 = default build, 3, 4 = libband_hip_pa{3,4}.so)
# - chain parity on pa3, then batch-24 kernel sums alternating the three
# builds on one box (each its own tuner), and every chain form per build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05al
mkdir -p $O
BAND_HIP_LIB_VARIANT=pa3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_chain_gpu.py > $O/tests_chain_pa3.log 2>&1 || exit 1
for r in 1 2; do
  for v in "" pa3 pa4; do
    BAND_HIP_LIB_VARIANT=$v BAND_HIP_TUNE_FILE=$O/tune_${v:-pa2}_r$r.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_${v:-pa2}_r$r.txt 2>&1 || exit 2
  done
done
for v in "" pa3 pa4; do
  BAND_HIP_LIB_VARIANT=$v timeout -k 10 200 python -u tools/chain_bench.py --batch 24 --iters 20 --px 1,2,4,4p,1w8,1w16,t > $O/chain_${v:-pa2}.txt 2>&1 || exit 3
done
echo done
