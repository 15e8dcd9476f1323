#!/bin/bash
# round 5: the chain kernel's depthwise phase with column reuse (group-1/2
# lanes take group 0's tap dwords by ds_bpermute; filter bytes from the tap
# table row) - chain parity, then the same-box batch-24 kernel-sum A/B
# against the r05f tree (abtree/r05f), alternating, each tree its own tuner
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05aj
mkdir -p $O
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chain_gpu.py > $O/tests_chain.log 2>&1 || exit 1
for r in 1 2; do
  (cd abtree/r05f && BAND_HIP_TUNE_FILE=$R/$O/tune_a_r$r.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400) > $O/breakdown_a_r$r.txt 2>&1 || exit 3
  BAND_HIP_TUNE_FILE=$R/$O/tune_b_r$r.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_b_r$r.txt 2>&1 || exit 4
done
(cd abtree/r05f && timeout -k 10 120 python -u tools/chain_bench.py --batch 24 --iters 20) > $O/chain_a.txt 2>&1 || exit 5
timeout -k 10 120 python -u tools/chain_bench.py --batch 24 --iters 20 > $O/chain_b.txt 2>&1 || exit 6
echo done
