#!/bin/bash
# round 5: the RGB stem with its constants staged in LDS (default) against
# the scalar-cache form (hint 6) - parity, then B = 1 / 24 / 32 interleaved x2,
# then the batch-24 mix breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem" > $O/tests_stem.log 2>&1 || exit 1
for r in 1 2; do
  for h in 4 6; do
    timeout -k 10 120 python3 -u tools/mfma_layer_bench.py --batches 1,24,32 --hint $h --only stem > $O/stem_h${h}_r$r.txt 2>&1 || exit 2
  done
done
timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_b24.txt 2>&1 || exit 3
echo done
