#!/bin/bash
# round 5: the column-blend bilinear resize with R output rows per
# workgroup (BH_RESIZE_ROWS_PER_WG 1 = the previous kernel's shape, 4 =
# default, 8) - glue / DeepLab parity, then DeepLab's batch-24 breakdown
# alternating the three on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05at
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_glue_gpu.py > $O/tests_glue.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_config_parity_gpu.py tests/test_executor_gpu.py -k "deeplab or resize" > $O/tests_deeplab.log 2>&1 || exit 2
for r in 1 2; do
  for v in 1 4 8; do
    BH_RESIZE_ROWS_PER_WG=$v timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 --top 400 --models deeplab_v3_mobilenet_v2 > $O/breakdown_rpw${v}_r$r.txt 2>&1 || exit 3
  done
done
echo done
