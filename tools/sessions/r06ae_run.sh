#!/bin/bash
# round 6: the persistent LDS stem (tile loop, next tile's rows prefetched
# into registers): stem parity, then the stem at batch 32 / 24 over
# BH_STEM_WG_PER_CU (8 = one tile per workgroup at these sizes, the old
# schedule), two rounds interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06ae
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "conv_stem or first_layer" > gpurun_out/r06ae/tests.log 2>&1 || { tail -30 gpurun_out/r06ae/tests.log; exit 1; }
tail -3 gpurun_out/r06ae/tests.log
for r in 1 2; do
  for b in 32 24; do
    for v in 8 1 2 3 4 6; do
      echo "round $r batch $b per_cu $v: $(BH_STEM_WG_PER_CU=$v timeout -k 10 120 python tools/layer_bench.py --only stem --batch $b --iters 50 | head -1)" \
        | tee -a gpurun_out/r06ae/stem.txt || exit 1
    done
  done
done
echo done
