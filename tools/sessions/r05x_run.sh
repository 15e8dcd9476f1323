#!/bin/bash
# round 5 final tree, one call (the pool is congested): the whole GPU suite
# and smoke(); the LDS stem with 1 / 2 pixels per thread (B = 24 / 32,
# interleaved); the batch-24 breakdown with the tuner log (the stem fused
# into the first tile chain, its records in LDS); the profile set r05y
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
for px in 1 2 1 2; do
  BH_STEM_PX=$px timeout -k 10 120 python3 -u tools/mfma_layer_bench.py --batches 24,32 --only stem >> $O/stem_px$px.txt 2>&1 || exit 3
done
BAND_HIP_TUNE_LOG=1 timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_b24.txt 2> $O/tunelog_b24.txt || exit 4
bash tools/profile_r05.sh r05y > $O/profile.log 2>&1 || exit 5
echo done
