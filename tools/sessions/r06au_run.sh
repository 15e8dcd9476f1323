#!/bin/bash
# round 6: the default line replaying the committed profile set's tuner
# decisions (profiles/r06an_tune.txt, matched through the PMC file's kernel
# tag) against --fresh-tuning: value, p99 and the roofline traffic ratio
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06au
mkdir -p $O
for v in replay_r1 fresh_r1 replay_r2; do
  a=""; [ "${v%%_*}" = fresh ] && a="--fresh-tuning"
  timeout -k 10 420 python -u bench.py $a > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 - $O/$v.json $v <<'PY' | tee -a $O/summary.txt
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]; lp = d.get("latency_point") or {}
print("%s: %.0f p99 %.2f | %s %.4f traffic/alg %s | latency point %.0f p99 %.2f | %s" % (
    sys.argv[2], d["value"], d["p99_job_latency_ms"], r["kernel"], r["frac"], r.get("traffic_over_algorithmic"),
    lp.get("value", 0), lp.get("p99_job_latency_ms", 0), d["config"].get("fusion_tuning")))
PY
done
echo done
