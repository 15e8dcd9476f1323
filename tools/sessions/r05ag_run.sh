#!/bin/bash
# round 5: the deep-issue phase A in the 64-pixel chain forms (6 depthwise
# channel groups per round instead of 2) - chain parity, per-chain times at
# B = 24 (plain vs deep, 64- and 32-pixel forms), the batch-24 mix kernel sum
# with the tuner free to take it, interleaved x2 against the form set without it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ag
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chain_gpu.py > $O/tests_chain.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/chain_bench.py --batch 24 --px "4,4d,2,2d" > $O/chain_deep_b24.txt 2>&1 || exit 2
for r in 1 2; do
  BAND_HIP_TUNE_LOG=1 timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_default_r$r.txt 2> $O/tunelog_r$r.txt || exit 3
  BAND_HIP_FUSION=nodeep timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_nodeep_r$r.txt 2>&1 || exit 4
done
echo done
