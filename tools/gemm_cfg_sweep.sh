#!/usr/bin/env bash
# A-B of conv_gemm_kernel configurations (BH_GEMM_CFG) on the deep / wide
# batched 1x1 shapes of tools/gemm_bench.py; parity of each vs conv_mfma_kernel
# is checked inside gemm_bench.  usage: tools/gemm_cfg_sweep.sh <out prefix> [cfgs]
set -u
P=${1:?prefix}
CFGS=${2:-"0 1 2 3 4 5 6 7"}
for c in $CFGS; do
  echo "== BH_GEMM_CFG=$c" >> "$P.txt"
  BH_GEMM_CFG=$c timeout -k 10 120 python3 tools/gemm_bench.py >> "$P.txt" 2>&1 || exit 1
done
