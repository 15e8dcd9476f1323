#!/bin/bash
# round 5: batch-1 MobileNetV2 (C2's job) on the final tree - per-launch
# breakdown and the chain tuner's measured forms
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ac
mkdir -p $O
BAND_HIP_TUNE_LOG=1 timeout -k 10 300 python -u tools/mix_breakdown.py --batch 1 --top 400 > $O/breakdown_b1.txt 2> $O/tunelog_b1.txt || exit 1
echo done
