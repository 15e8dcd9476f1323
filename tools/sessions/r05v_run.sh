#!/bin/bash
# round 5: the LDS-staged stem with 1 or 2 pixels per thread - parity, B = 24
# / 32 interleaved x2, the batch-24 mix breakdown and the tuner's decision on
# the stem fused into the first tile chain (its channel records now in LDS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_chain_gpu.py -k "stem" > $O/tests_stem.log 2>&1 || exit 1
for r in 1 2; do
  for px in 1 2; do
    BH_STEM_PX=$px timeout -k 10 120 python3 -u tools/mfma_layer_bench.py --batches 24,32 --only stem > $O/stem_px${px}_r$r.txt 2>&1 || exit 2
  done
done
BAND_HIP_TUNE_LOG=1 timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_b24.txt 2> $O/tunelog_b24.txt || exit 3
echo done
