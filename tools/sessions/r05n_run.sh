#!/bin/bash
# round 5: the chain kernel's VALU / split variants as compile-time
# instantiations (the default one carries none of their code) - chain and
# stem parity, then the same-box batch-24 kernel-sum A/B against the round-4
# tree (its own tuner, and its choices replayed on this tree)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05n
mkdir -p $O
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chain_gpu.py > $O/tests_chain.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem" > $O/tests_stem.log 2>&1 || exit 2
for r in 1 2; do
  (cd abtree/r04 && BAND_HIP_TUNE_FILE=$R/$O/tune_r04.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400) > $O/breakdown_r04tree_r$r.txt 2>&1 || exit 3
  python3 tools/tune_translate.py $O/tune_r04.txt $O/tune_r04_as_now_r$r.txt > /dev/null || exit 4
  BAND_HIP_TUNE_FILE=$R/$O/tune_r04_as_now_r$r.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_now_r04choices_r$r.txt 2>&1 || exit 5
  BAND_HIP_TUNE_LOG=1 timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_now_r$r.txt 2> $O/tunelog_now_r$r.txt || exit 6
done
echo done
