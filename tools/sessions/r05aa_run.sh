#!/bin/bash
# round 5: the fused stem prologue on MFMA - parity (forced on the C3 models
# and ragged sizes, stem kernels), then the batch-24 breakdown with the
# tuner's fused-vs-separate decision
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_chain_gpu.py -k "stem" > $O/tests_stem.log 2>&1 || exit 1
BAND_HIP_TUNE_LOG=1 timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_b24.txt 2> $O/tunelog_b24.txt || exit 2
echo done
