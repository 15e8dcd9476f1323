#!/bin/bash
# round 5, part 1: parity of this round's kernels (conv_gemm_big, stem on
# MFMA, chain split + VALU depthwise forms, coalescer), then the MobileNetV2
# Conv2D MFMA-i8 roofline micro-benchmark at B = 1 / 32 / 256 (routed, and
# the big GEMM forced) and the MobileNetV2 batch-1 breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05h
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py -k "gemm or stem" > $O/tests_kernels.log 2>&1 || exit 1
timeout -k 10 500 $T tests/test_chain_gpu.py -k "split or valu" > $O/tests_chain.log 2>&1 || exit 1
timeout -k 10 300 $T tests/test_coalescer_gpu.py > $O/tests_coalescer.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/mfma_layer_bench.py --json $O/mfma_layers.json > $O/mfma_layers.txt 2>&1 || exit 2
timeout -k 10 300 python -u tools/mfma_layer_bench.py --batches 32,256 --hint 3 --json $O/mfma_layers_big.json > $O/mfma_layers_big.txt 2>&1 || exit 3
timeout -k 10 200 python -u tools/mix_breakdown.py --batch 1 --models mobilenet_v2 --top 30 > $O/breakdown_mnv2_b1.txt 2>&1 || exit 4
echo done
