#!/bin/bash
# round 5: the staged-row LDS stem with its 32 channels split over 2 / 4
# workgroups per pixel block (BH_STEM_MIN_WG 2352 / 4704) against one
# (default) - stem parity under the split, then batch-24 breakdowns
# alternating on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ax
mkdir -p $O
BH_STEM_MIN_WG=4704 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k stem > $O/tests_stem_split.log 2>&1 || exit 1
for r in 1 2; do
  for v in 512 2352 4704; do
    BH_STEM_MIN_WG=$v BAND_HIP_TUNE_FILE=$O/tune_${v}_r$r.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_mw${v}_r$r.txt 2>&1 || exit 2
  done
done
echo done
