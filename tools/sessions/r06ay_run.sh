#!/bin/bash
# round 6: C5's intermittent p99 tail - where the slow (> 10 ms) jobs fall
# (bench.py latency_tail: per model / worker, clusters in arrival order);
# five repeats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06ay
mkdir -p $O
for r in 1 2 3 4 5 6; do
  timeout -k 10 300 python3 bench.py --model mix_c5 --scheduler shortest_expected_latency --job-batch 1 --rate 4200 --no-cpu-baseline > $O/c5_r$r.json 2> $O/c5_r$r.err || exit 1
  python3 -c "import json;d=json.load(open('$O/c5_r$r.json'));print('c5 round $r', round(d['value']), round(d['p50_job_latency_ms'],2), round(d['p99_job_latency_ms'],2), json.dumps(d.get('latency_tail')))" | tee -a $O/summary.txt
done
echo done
