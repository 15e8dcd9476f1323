#!/bin/bash
# round 6: the committed default line, three more repeats on one box (the
# run-to-run spread the driver's single run samples from)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06aw
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 420 python -u bench.py > $O/bench_r$r.json 2> $O/bench_r$r.err || { tail -5 $O/bench_r$r.err; exit 1; }
  python3 - $O/bench_r$r.json $r <<'PY' | tee -a $O/summary.txt
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]; lp = d.get("latency_point") or {}; b = d["band_one_job_per_pass"]
print("round %s: %.0f p99 %.2f | %s %.4f x%.3f | band48 %.0f band12 %.0f | latency point %.0f p99 %.2f" % (
    sys.argv[2], d["value"], d["p99_job_latency_ms"], r["kernel"], r["frac"], r.get("traffic_over_algorithmic") or 0,
    b["value"], b["at_12_workers_per_gpu"]["value"], lp.get("value", 0), lp.get("p99_job_latency_ms", 0)))
PY
done
echo done
