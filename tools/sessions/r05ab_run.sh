#!/bin/bash
# round 5: conv_gemm_big_kernel below its routing bound - the batch-24
# PoseNet / MobileNetV2 / SSD 1x1 layers with the routed kernel (hint 0)
# against the big tile forced (hint 3) in each tile configuration
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ab
mkdir -p $O
F="posenet|960->|1280->|576->|320->"
for r in 1 2; do
  timeout -k 10 120 python3 -u tools/mfma_layer_bench.py --batches 16,24 --only "$F" > $O/routed_r$r.txt 2>&1 || exit 1
  for cfg in 2 3; do
    BH_GEMM_BIG_CFG=$cfg timeout -k 10 120 python3 -u tools/mfma_layer_bench.py --batches 16,24 --hint 3 --only "$F" > $O/big_cfg${cfg}_r$r.txt 2>&1 || exit 2
  done
done
echo done
