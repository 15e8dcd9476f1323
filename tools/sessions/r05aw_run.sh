#!/bin/bash
# round 5: the tile chain's depthwise taps by filter row / column (lane
# group 3 idle; default build) against taps 4s + g (libband_hip_tm0.so) -
# chain parity, tile-form times, then batch-24 kernel sums alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05aw
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_chain_gpu.py > $O/tests_chain.log 2>&1 || exit 1
for v in tm0 "" tm0 ""; do
  BAND_HIP_LIB_VARIANT=$v timeout -k 10 120 python -u tools/chain_bench.py --batch 24 --iters 30 --px t >> $O/chain_${v:-tm1}.txt 2>&1 || exit 2
done
for r in 1 2; do
  for v in tm0 ""; do
    BAND_HIP_LIB_VARIANT=$v BAND_HIP_TUNE_FILE=$O/tune_${v:-tm1}_r$r.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_${v:-tm1}_r$r.txt 2>&1 || exit 3
  done
done
echo done
