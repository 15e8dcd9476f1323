#!/bin/bash
# round 6: conv_gemm_kernel tile rule at batch 32 (the default job batch):
# BH_GEMM_CFG 0 (64x64 tiles below one chip of 128x128) against 1 (the
# 4-wave 128x128 / 128x64 / 64x128 rule), whole-mix breakdown, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06ar
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    BH_GEMM_CFG=$v timeout -k 10 400 python -u tools/mix_breakdown.py --batch 32 --top 400 > $O/b32_cfg${v}_r$r.txt 2>&1 || exit 1
    echo "round $r cfg $v: $(grep 'sum of kernel-only' $O/b32_cfg${v}_r$r.txt) | $(grep '^  conv_gemm_kernel' $O/b32_cfg${v}_r$r.txt)" | tee -a $O/summary.txt
  done
done
echo done
