#!/bin/bash
# round 6: how much the fusion tuner's per-process decisions move the
# default line: four fresh processes each record their decisions (a tune
# file of their own), then every decision set is replayed twice, interleaved
# (--no-cpu-baseline: the headline, Band-contract and latency-point lines)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06az
mkdir -p $O
for k in 1 2 3 4; do
  rm -f $O/tune_$k.txt
  BAND_HIP_TUNE_FILE=$O/tune_$k.txt timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/fresh_$k.json 2> $O/fresh_$k.err || { tail -5 $O/fresh_$k.err; exit 1; }
done
for r in 1 2; do
  for k in 1 2 3 4; do
    cp $O/tune_$k.txt $O/replay_scratch.txt
    BAND_HIP_TUNE_FILE=$O/replay_scratch.txt timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/replay_${k}_r$r.json 2> $O/replay_${k}_r$r.err || { tail -5 $O/replay_${k}_r$r.err; exit 1; }
  done
done
rm -f $O/replay_scratch.txt
python3 - <<'PY' | tee $O/summary.txt
import json
O = "gpurun_out/r06az"
def line(f):
    d = json.load(open(f)); lp = d.get("latency_point") or {}
    return "%.0f p99 %.2f | lp %.0f p99 %.2f | chain %.4f" % (d["value"], d["p99_job_latency_ms"], lp.get("value", 0),
                                                             lp.get("p99_job_latency_ms", 0), d["roofline"]["frac"])
for k in (1, 2, 3, 4):
    print("set %d fresh: %s" % (k, line("%s/fresh_%d.json" % (O, k))))
    for r in (1, 2):
        print("set %d replay r%d: %s" % (k, r, line("%s/replay_%d_r%d.json" % (O, k, r))))
PY
echo done
