#!/bin/bash
# round 5: the tile chain at 6 waves per SIMD (BH_TILE_WPE=6 build,
# libband_hip_tw6.so: 80 VGPRs, 4 spilled) against the default (95 VGPRs,
# 5 waves) - tile parity on tw6, tile-form times per chain, then batch-24
# kernel sums alternating the two builds on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05an
mkdir -p $O
BAND_HIP_LIB_VARIANT=tw6 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_chain_gpu.py > $O/tests_chain_tw6.log 2>&1 || exit 1
for v in "" tw6 "" tw6; do
  BAND_HIP_LIB_VARIANT=$v timeout -k 10 120 python -u tools/chain_bench.py --batch 24 --iters 30 --px t,tp > $O/chain_${v:-def}.txt 2>&1 || exit 2
done
for r in 1 2; do
  for v in "" tw6; do
    BAND_HIP_LIB_VARIANT=$v BAND_HIP_TUNE_FILE=$O/tune_${v:-def}_r$r.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_${v:-def}_r$r.txt 2>&1 || exit 3
  done
done
echo done
