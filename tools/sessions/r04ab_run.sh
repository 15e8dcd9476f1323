#!/usr/bin/env bash
# workers-per-GPU A-B at a fixed in-flight depth (interleaved, no CPU baseline)
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do
  i=0
  for v in "--workers-per-gpu 8" "--workers-per-gpu 4 --inflight 384" "--workers-per-gpu 6 --inflight 384" "--workers-per-gpu 8 --inflight 512"; do
    BANDX_REQUEST_RING_SLOTS=256 timeout -k 10 250 python3 bench.py --no-cpu-baseline --no-batch1 $v > $O/r04ab_v${i}_r$r.json 2> $O/r04ab_v${i}_r$r.err || exit 1
    i=$((i + 1))
  done
done
