#!/bin/bash
# round 5: conv_gemm_big_kernel with the epilogue constants staged in LDS and
# deeper K pipelines - parity, then every tile configuration at B = 256 on
# the high-intensity layers, and the routed micro-benchmark at B = 32 / 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or stem" > $O/tests_kernels.log 2>&1 || exit 1
for cfg in 1 2 3 4 5; do
  BH_GEMM_BIG_CFG=$cfg timeout -k 10 200 python3 -u tools/mfma_layer_bench.py --batches 256 --hint 3 --only "1280|1024|960->320" > $O/cfg$cfg.txt 2>&1 || exit 2
done
echo done
