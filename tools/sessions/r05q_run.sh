#!/bin/bash
# round 5: the RGB stem fused into the first tile chain - parity (forced,
# every C3 model, ragged sizes), the tuner's decision log, and the batch-24
# kernel-sum A/B (default vs BAND_HIP_FUSION=nostem, interleaved x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chain_gpu.py -k "stem" > $O/tests_stem.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_coalescer_gpu.py > $O/tests_coalescer.log 2>&1 || exit 2
for r in 1 2; do
  BAND_HIP_TUNE_LOG=1 timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_default_r$r.txt 2> $O/tunelog_default_r$r.txt || exit 3
  BAND_HIP_FUSION=nostem timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_nostem_r$r.txt 2>&1 || exit 4
done
echo done
