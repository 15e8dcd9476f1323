#!/bin/bash
# round 6: the default bench line with the latency_point side line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06z
mkdir -p $O
for r in 1 2; do
  timeout -k 10 400 python -u bench.py > $O/bench_default_r$r.json 2> $O/bench_default_r$r.err || exit 1
done
echo done
