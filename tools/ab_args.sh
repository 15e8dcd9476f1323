#!/usr/bin/env bash
# Interleaved A-B of bench.py argument variants.
# Usage: tools/ab_args.sh TAG ROUNDS "ARGS A" "ARGS B" ...   (outputs gpurun_out/TAG_v<i>_r<k>.json)
set -uo pipefail
TAG=$1; ROUNDS=$2; shift 2
O=gpurun_out; mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  i=0
  for v in "$@"; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline $v > $O/${TAG}_v${i}_r$r.json 2> $O/${TAG}_v${i}_r$r.err || exit $?
    echo "$TAG v$i ($v) round $r: $(python3 -c "import json;d=json.load(open('$O/${TAG}_v${i}_r$r.json'));print(round(d['value']), d['p99_job_latency_ms'])")"
    i=$((i+1))
  done
done
