#!/bin/bash
# round 6: the multi-row column-blend resize with 24-bit multiplies and the shift rounding (DeepLab's batched logits
# upsample): parity, then DeepLab's batch-32 / 24 breakdown over
# BH_RESIZE_ROWS (1 = one row per workgroup, the old schedule; 0 = the
# launcher's choice), two rounds interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06ai
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_glue_gpu.py \
  -k "resize" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for b in 32 24; do
    for v in 1 0; do
      BH_RESIZE_ROWS=$v timeout -k 10 300 python tools/mix_breakdown.py --models deeplab_v3_mobilenet_v2 --batch $b \
        --iters 20 --top 60 > $O/dl_b${b}_rows${v}_r$r.txt 2>&1 || { tail -5 $O/dl_b${b}_rows${v}_r$r.txt; exit 1; }
      echo "round $r batch $b rows $v: $(grep -m1 'graph replay' $O/dl_b${b}_rows${v}_r$r.txt | cut -c1-90) | $(grep -m1 ' 68 resize' $O/dl_b${b}_rows${v}_r$r.txt)" | tee -a $O/summary.txt
    done
  done
done
echo done
