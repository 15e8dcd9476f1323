#!/bin/bash
# round 5: six default bench lines back to back on one box, with per-model
# latency percentiles, to catch the run-to-run outlier (~104k, p99 ~12 ms)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05au
mkdir -p $O
for r in 1 2 3 4 5 6; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_r$r.json 2> $O/bench_r$r.err || exit $r
done
echo done
