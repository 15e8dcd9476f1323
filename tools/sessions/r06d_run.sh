#!/bin/bash
# round 6: per-phase shader-clock stamps of chain_kernel's few-pixel forms
# at batch 24 (where the stage form did not pay) and batch 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06d
mkdir -p $O
for f in 1w8 1w16 1 2; do
  timeout -k 10 120 python -u tools/tile_probe.py --batch 24 --only 3,4,5,6,7,8,9,10,11 --raster $f > $O/probe_b24_$f.txt 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/tile_probe.py --batch 1 --only 6,7,8,9,10,11 --raster 1w8 > $O/probe_b1_1w8.txt 2>&1 || exit 2
echo done
