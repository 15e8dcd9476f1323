#!/bin/bash
# round 6: the stage chain form - parity, then chain times at batch 24 / 1
# against the raster forms (and the round-5 fused_chain.hip build for the
# refactor of phase A into chain_dw.hpp), then the batch-24 mix breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chain_gpu.py -k "stage" > $O/tests_stage.log 2>&1 || { tail -30 $O/tests_stage.log; exit 1; }
tail -3 $O/tests_stage.log
F=1,1w8,1w16,g1w4,g1w8,g2w4,g2w8,g1w4s2,g1w8s2,g2w8s2,g1w8s4,g1w4s4,g1w8s8
BAND_HIP_LIB_VARIANT=r05chain timeout -k 10 120 python -u tools/chain_bench.py --batch 24 --iters 30 --px 1,2,4,1w8,1w16 > $O/chain_b24_r05chain.txt 2>&1 || exit 2
timeout -k 10 200 python -u tools/chain_bench.py --batch 24 --iters 30 --px 1,2,4,1w8,1w16 > $O/chain_b24_new_oldforms.txt 2>&1 || exit 3
timeout -k 10 200 python -u tools/chain_bench.py --batch 24 --iters 30 --px $F > $O/chain_b24.txt 2>&1 || exit 4
timeout -k 10 200 python -u tools/chain_bench.py --batch 1 --iters 30 --px $F > $O/chain_b1.txt 2>&1 || exit 5
BAND_HIP_TUNE_LOG=1 BAND_HIP_TUNE_FILE=$O/tune_b24.txt timeout -k 10 400 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_b24.txt 2> $O/tunelog_b24.txt || exit 6
BAND_HIP_FUSION=nostage BAND_HIP_TUNE_FILE=$O/tune_b24_nostage.txt timeout -k 10 400 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_b24_nostage.txt 2>&1 || exit 7
echo done
