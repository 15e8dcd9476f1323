#!/bin/bash
# round 5 final tree (one pixel per thread in the LDS stem): stem parity, the
# batch-24 breakdown, and the profile set r05y2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_chain_gpu.py -k "stem" > $O/tests_stem.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_b24.txt 2>&1 || exit 2
bash tools/profile_r05.sh r05y2 > $O/profile.log 2>&1 || exit 3
echo done
