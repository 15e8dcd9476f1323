#!/bin/bash
# round 5: conv_gemm_big_kernel parity, then the MobileNetV2 Conv2D MFMA-i8
# roofline micro-benchmark at B = 1 / 32 / 256: the routed kernels, and the
# big GEMM / the 128-tile GEMM forced
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/mfma_layer_bench.py --json $O/mfma_layers.json > $O/mfma_layers.txt 2>&1 || exit 2
timeout -k 10 300 python -u tools/mfma_layer_bench.py --batches 32,256 --hint 3 --json $O/mfma_layers_big.json > $O/mfma_layers_big.txt 2>&1 || exit 3
timeout -k 10 300 python -u tools/mfma_layer_bench.py --batches 32,256 --hint 2 > $O/mfma_layers_gemm128.txt 2>&1 || exit 4
for cfg in 2 3 4; do
  BH_GEMM_BIG_CFG=$cfg timeout -k 10 300 python -u tools/mfma_layer_bench.py --batches 256 --hint 3 > $O/mfma_big_cfg$cfg.txt 2>&1 || exit 5
done
echo done
