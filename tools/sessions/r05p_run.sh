#!/bin/bash
# round 5: host cores per GPU - spinning waits vs sleep-then-spin
# (BAND_HIP_SYNC=adaptive, sleeping 0.7 / 0.85 of the expected wait),
# interleaved x2 on the C3 headline, then Band's own contract (48 workers)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05p
mkdir -p $O
export BAND_HIP_TUNE_FILE=$O/tune.txt
B="--no-cpu-baseline --no-roofline --no-batch1 --no-single-engine"
timeout -k 10 400 python bench.py $B --steps 4 --warmup 2 > $O/warm.json 2> $O/warm.err || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/bench_spin_r$r.json 2> $O/bench_spin_r$r.err || exit 2
  BAND_HIP_SYNC=adaptive timeout -k 10 300 python bench.py $B > $O/bench_ad70_r$r.json 2> $O/bench_ad70_r$r.err || exit 3
  BAND_HIP_SYNC=adaptive BAND_HIP_SYNC_SLEEP=0.85 timeout -k 10 300 python bench.py $B > $O/bench_ad85_r$r.json 2> $O/bench_ad85_r$r.err || exit 4
done
BAND_HIP_SYNC=adaptive timeout -k 10 300 python bench.py --job-batch 1 --workers-per-gpu 48 --steps 10 --warmup 3 $B > $O/band1_ad70.json 2> $O/band1_ad70.err || exit 5
echo done
