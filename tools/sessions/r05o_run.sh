#!/bin/bash
# round 5: the C3 headline - default (spinning waits) vs the completion
# poller (BAND_HIP_SYNC=poller), interleaved x2, then Band's own contract
# (max_job_batch 1, 48 workers, the coalescer) with both waits
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05o
mkdir -p $O
export BAND_HIP_TUNE_FILE=$O/tune.txt
B="--no-cpu-baseline --no-roofline --no-batch1 --no-single-engine"
timeout -k 10 400 python bench.py $B --steps 4 --warmup 2 > $O/warm.json 2> $O/warm.err || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/bench_default_r$r.json 2> $O/bench_default_r$r.err || exit 2
  BAND_HIP_SYNC=poller timeout -k 10 300 python bench.py $B > $O/bench_poller_r$r.json 2> $O/bench_poller_r$r.err || exit 3
done
for s in spin poller; do
  BAND_HIP_SYNC=$s timeout -k 10 300 python bench.py --job-batch 1 --workers-per-gpu 48 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-batch1 --no-single-engine > $O/band1_$s.json 2> $O/band1_$s.err || exit 4
done
echo done
