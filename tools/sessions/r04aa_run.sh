#!/usr/bin/env bash
# hardware queues / workers A-B on the final tree (interleaved, no CPU baseline)
export TMPDIR=/tmp
O=gpurun_out
i=0
for r in 1 2; do
  for v in "--hw-queues 4" "--hw-queues 8" "--hw-queues 8 --workers-per-gpu 12" "--hw-queues 6 --workers-per-gpu 8"; do
    timeout -k 10 250 python3 bench.py --no-cpu-baseline --no-batch1 $v > $O/r04aa_v$((i % 4))_r$r.json 2> $O/r04aa_v$((i % 4))_r$r.err || exit 1
    i=$((i + 1))
  done
done
