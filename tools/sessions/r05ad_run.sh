#!/bin/bash
# round 5: with waits sleeping, does the C3 headline gain from a second
# request submitter?  BANDX_DRIVER_LANES 1 (default) vs 2, interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ad
mkdir -p $O
export BAND_HIP_TUNE_FILE=$O/tune.txt
B="--no-cpu-baseline --no-roofline --no-batch1 --no-single-engine"
timeout -k 10 400 python bench.py $B --steps 4 --warmup 2 > $O/warm.json 2> $O/warm.err || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/lanes1_r$r.json 2> $O/lanes1_r$r.err || exit 2
  BANDX_DRIVER_LANES=2 timeout -k 10 300 python bench.py $B > $O/lanes2_r$r.json 2> $O/lanes2_r$r.err || exit 3
done
echo done
