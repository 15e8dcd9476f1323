#!/bin/bash
# round 5: where the column-reuse chain forms spend their time - every form
# of every MobileNetV2 chain at batch 24 (tools/chain_bench.py), and the
# per-phase shader-clock stamps of the raster forms (tools/tile_probe.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ak
mkdir -p $O
timeout -k 10 300 python -u tools/chain_bench.py --batch 24 --iters 20 > $O/chain_bench_b24.txt 2>&1 || exit 1
for f in 1w8 1 2 4; do
  timeout -k 10 120 python -u tools/tile_probe.py --batch 24 --raster $f > $O/probe_$f.txt 2>&1 || exit 2
done
echo done
