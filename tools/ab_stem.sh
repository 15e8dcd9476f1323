#!/usr/bin/env bash
# A-B of the stem's channel split (BH_STEM_MIN_WG: workgroups the launcher
# aims for by splitting the output channels over grid.y) on the batch-24
# MobileNetV2 pass; parity of the stem under the widest split first.
set -uo pipefail
O=gpurun_out; mkdir -p $O
BH_STEM_MIN_WG=4800 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "stem or conv" --timeout 120 --timeout-method thread > $O/stem_tests.log 2>&1 || exit $?
for rep in 1 2; do
  for w in 512 2400 4800; do
    BH_STEM_MIN_WG=$w timeout -k 10 120 python tools/mix_breakdown.py --batch 24 --models mobilenet_v2,posenet_mobilenet_v1 --top 4 > $O/stem_w${w}_r$rep.txt 2>&1 || exit $?
  done
done
echo stem ab done
