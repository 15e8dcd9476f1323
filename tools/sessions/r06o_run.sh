#!/bin/bash
# round 6: the chain tuner's own measurements at batch 1 (MobileNetV2), to
# see why the 7x7 chains stay unfused there
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06o
mkdir -p $O
BAND_HIP_TUNE_LOG=1 timeout -k 10 200 python -u tools/mix_breakdown.py --batch 1 --models mobilenet_v2 --top 60 > $O/mnv2_b1.txt 2> $O/mnv2_b1_tune.log || exit 1
echo done
