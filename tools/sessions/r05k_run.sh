#!/bin/bash
# round 5: the 2-workgroups-per-CU big-GEMM default - parity, the routed
# MFMA micro-benchmark at B = 1 / 32 / 256, then the batch-24 kernel-sum A/B
# of the chain tuner's form sets (default / nosplit / novalu, interleaved x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or stem" > $O/tests_kernels.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/mfma_layer_bench.py --batches 1,32,256 --json $O/mfma_layers.json > $O/mfma_layers.txt 2>&1 || exit 2
for r in 1 2; do
  for arm in nosplit novalu default; do
    if [ $arm = default ]; then unset BAND_HIP_FUSION; else export BAND_HIP_FUSION=$arm; fi
    timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 > $O/breakdown_${arm}_r$r.txt 2>&1 || exit 3
  done
done
echo done
