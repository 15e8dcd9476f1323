#!/bin/bash
# round 5 final tree: where a workgroup of the biggest chains spends its
# clocks (s_memtime stamps at the phase boundaries) - the 112x112 x 32 tile
# chain and the 56x56 x 144 residual raster chain at B = 24
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05af
mkdir -p $O
timeout -k 10 120 python3 -u tools/tile_probe.py --batch 24 --only 0,1,2 > $O/tile_probe_b24.txt 2>&1 || exit 1
timeout -k 10 120 python3 -u tools/tile_probe.py --batch 24 --only 1,2,6 --raster 4 > $O/raster_probe_b24.txt 2>&1 || exit 2
echo done
