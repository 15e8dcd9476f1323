#!/bin/bash
# round 5: where the +70 us of batch-24 mix kernel time since round 4 comes
# from - full launch lists of the round-4 tree and this tree, the round-4
# tuner's chain choices replayed on this tree's kernels, and this tree's
# tuner log (every chain form measured)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05m
mkdir -p $O
R=$(pwd)
for r in 1 2; do
  (cd abtree/r04 && BAND_HIP_TUNE_FILE=$R/$O/tune_r04.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400) > $O/breakdown_r04tree_r$r.txt 2>&1 || exit 1
  python3 tools/tune_translate.py $O/tune_r04.txt $O/tune_r04_as_now_r$r.txt > /dev/null || exit 2
  BAND_HIP_TUNE_FILE=$R/$O/tune_r04_as_now_r$r.txt timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_now_r04choices_r$r.txt 2>&1 || exit 3
  BAND_HIP_TUNE_LOG=1 timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 > $O/breakdown_now_r$r.txt 2> $O/tunelog_now_r$r.txt || exit 4
done
echo done
