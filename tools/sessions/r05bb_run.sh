#!/bin/bash
# round 5: channel tiles per round of the x-stationary 1x1 GEMMs in the
# chain kernel's default forms (TTC 2 = default; 3 / 4 =
# libband_hip_ttc{3,4}.so, built from a copy with TTC a build switch) -
# chain forms and batch-24 kernel sums alternating on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05bb
mkdir -p $O
for v in "" ttc3 ttc4; do
  BAND_HIP_LIB_VARIANT=$v timeout -k 10 120 python -u tools/chain_bench.py --batch 24 --iters 30 --px 1,2,4,1w8,1w16 > $O/chain_${v:-ttc2}.txt 2>&1 || exit 1
done
for r in 1 2; do
  for v in "" ttc3 ttc4; do
    BAND_HIP_LIB_VARIANT=$v BAND_HIP_TUNE_FILE=$O/tune_${v:-ttc2}_r$r.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_${v:-ttc2}_r$r.txt 2>&1 || exit 2
  done
done
echo done
