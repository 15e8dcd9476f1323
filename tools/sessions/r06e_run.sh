#!/bin/bash
# round 6: conv_gemm_big with 128 x 128 wave tiles (one wave per SIMD,
# 256 x 256 workgroup tiles: BH_GEMM_BIG_CFG 6 / 7) and 128 x 64 (8) against
# the routed configuration (3), MobileNetV2 / PoseNet GEMM layers at B = 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06e
mkdir -p $O
L='7 960->160|7 960->320|7 320->1280|7 160->960|posenet|14 576->96'
for cfg in 3 6 7 8; do
  BH_GEMM_BIG_CFG=$cfg timeout -k 10 300 python -u tools/mfma_layer_bench.py --batches 256 --hint 3 --only "$L" > $O/mfma_cfg$cfg.txt 2>&1 || exit 1
done
echo done
