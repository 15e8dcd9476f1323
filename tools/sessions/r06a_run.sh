#!/bin/bash
# round 6, first call: the round-5 tree on a fresh box - default bench, the
# headline at fewer requests in flight (tail latency), and Band's own
# contract (job batch 1, backend coalescer) at 8 / 12 / 16 workers per GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
for inf in 192 240 288; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --inflight $inf --no-cpu-baseline --no-roofline --no-batch1 \
    > $O/bench_inf$inf.json 2> $O/bench_inf$inf.err || exit 2
done
for w in 8 12 16; do
  for wt in 100 300; do
    BAND_HIP_COALESCE_WAIT_US=$wt timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --job-batch 1 --workers-per-gpu $w \
      --no-cpu-baseline --no-roofline --no-batch1 > $O/band1_w${w}_wait$wt.json 2> $O/band1_w${w}_wait$wt.err || exit 3
  done
done
echo done
