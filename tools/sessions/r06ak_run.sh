#!/bin/bash
# round 6: fewer hardware queues per process than HIP's 4 (after r06aj: 8 / 16 lose)
# for the whole default line: the headline, Band's one-job-per-pass
# contract at 48 and 12 workers per GPU (12-48 concurrent batch-1 passes
# over 4 queues) and the latency point; two rounds interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06ak
mkdir -p $O
for r in 1 2; do
  for q in 4 2 3; do
    timeout -k 10 420 python3 bench.py --no-cpu-baseline --no-roofline --hw-queues $q > $O/q${q}_r$r.json 2> $O/q${q}_r$r.err || { tail -5 $O/q${q}_r$r.err; exit 1; }
    python3 - $O/q${q}_r$r.json $q $r <<'PY' | tee -a $O/summary.txt
import json, sys
d = json.load(open(sys.argv[1]))
b = d.get("band_one_job_per_pass") or {}
b12 = b.get("at_12_workers_per_gpu") or {}
lp = d.get("latency_point") or {}
print("q %s round %s: headline %.0f p99 %.2f | band48 %.0f p99 %.2f | band12 %.0f p99 %.2f | latency point %.0f p99 %.2f" % (
    sys.argv[2], sys.argv[3], d["value"], d["p99_job_latency_ms"], b.get("value", 0), b.get("p99_job_latency_ms", 0),
    b12.get("value", 0), b12.get("p99_job_latency_ms", 0), lp.get("value", 0), lp.get("p99_job_latency_ms", 0)))
PY
  done
done
echo done
