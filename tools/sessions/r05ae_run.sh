#!/bin/bash
# round 5: hardware queues with sleeping waits - the C3 headline at 4 (default)
# / 8 queues with 8 workers and 8 queues with 12 workers, interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ae
mkdir -p $O
export BAND_HIP_TUNE_FILE=$O/tune.txt
B="--no-cpu-baseline --no-roofline --no-batch1 --no-single-engine"
timeout -k 10 400 python bench.py $B --steps 4 --warmup 2 > $O/warm.json 2> $O/warm.err || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/q4w8_r$r.json 2> $O/q4w8_r$r.err || exit 2
  timeout -k 10 300 python bench.py $B --hw-queues 8 > $O/q8w8_r$r.json 2> $O/q8w8_r$r.err || exit 3
  timeout -k 10 300 python bench.py $B --hw-queues 8 --workers-per-gpu 12 > $O/q8w12_r$r.json 2> $O/q8w12_r$r.err || exit 4
done
echo done
