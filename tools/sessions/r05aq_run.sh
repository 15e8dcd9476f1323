#!/bin/bash
# round 5, final tree (r05i): two more default bench lines, untraced, to
# place the r05i final line (104.5k, p99 11.3 ms after the PMC passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05aq
mkdir -p $O
for r in 1 2; do
  timeout -k 10 500 python3 bench.py > $O/bench_r$r.json 2> $O/bench_r$r.err || exit $r
done
echo done
