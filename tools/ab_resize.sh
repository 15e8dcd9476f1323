#!/usr/bin/env bash
# Parity of the int8 RESIZE_BILINEAR launchers, then an A-B of the
# column-blend row kernel against the byte-blend row kernel (BH_RESIZE_ROWS=1)
# on DeepLab's batch-24 pass.
set -uo pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_glue_gpu.py tests/test_config_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/resize_tests.log 2>&1 || exit $?
echo tests done
for rep in 1 2; do
  for m in rows cols; do
    if [ $m = rows ]; then export BH_RESIZE_ROWS=1; else unset BH_RESIZE_ROWS; fi
    timeout -k 10 120 python tools/mix_breakdown.py --batch 24 --models deeplab_v3_mobilenet_v2 --top 6 > $O/resize_${m}_r$rep.txt 2>&1 || exit $?
  done
done
echo resize ab done
