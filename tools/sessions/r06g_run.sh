#!/bin/bash
# round 6: headline defaults, second sweep around job batch 32 with the
# pass-size policy (in flight x pass target x job batch), alternating twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06g
mkdir -p $O
for r in 1 2; do
  for v in "288 600 32" "320 700 32" "384 600 32" "384 700 40" "224 600 24"; do
    set -- $v
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --inflight $1 --pass-target-us $2 --job-batch $3 --no-cpu-baseline --no-roofline --no-batch1 \
      > $O/bench_inf$1_pt$2_jb$3_r$r.json 2> $O/bench_inf$1_pt$2_jb$3_r$r.err || exit 1
  done
done
echo done
