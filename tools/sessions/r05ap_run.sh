#!/bin/bash
# round 5: the LDS stem with its input rows staged in LDS by 16-byte loads
# (default build) against per-pixel window loads (libband_hip_r0.so,
# BH_STEM_ROWS=0) - stem, batched and whole-model parity, then batch-24
# kernel sums alternating the two builds on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ap
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k stem > $O/tests_stem.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_job_batch_gpu.py tests/test_config_parity_gpu.py > $O/tests_models.log 2>&1 || exit 2
for r in 1 2; do
  for v in r0 ""; do
    BAND_HIP_LIB_VARIANT=$v BAND_HIP_TUNE_FILE=$O/tune_${v:-rows}_r$r.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_${v:-rows}_r$r.txt 2>&1 || exit 3
  done
done
echo done
