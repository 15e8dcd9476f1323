#!/usr/bin/env bash
# A-B of the block-diagonal MFMA depthwise form against the VALU run / dot
# forms on the batch-24 C3 mix: standalone depthwise layers (chain fusion off,
# so every depthwise layer is its own launch) and the default fused tree.
set -uo pipefail
O=gpurun_out; mkdir -p $O
for fu in nochain default; do
  for dw in mfma valu; do
    if [ $fu = nochain ]; then export BAND_HIP_FUSION=nochain; else unset BAND_HIP_FUSION; fi
    if [ $dw = valu ]; then export BH_DW_MFMA_MIN_TILES=1000000000000; else unset BH_DW_MFMA_MIN_TILES; fi
    timeout -k 10 150 python tools/mix_breakdown.py --batch 24 --top 0 > $O/dwab_${fu}_${dw}.txt 2>&1 || exit $?
  done
done
echo dw ab done
