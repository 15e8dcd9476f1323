#!/usr/bin/env bash
# Interleaved A-B of bench.py under environment variants.
# Usage: tools/ab_env.sh TAG ROUNDS "VAR=a VAR2=b" "VAR=c" ...   (outputs gpurun_out/TAG_v<i>_r<k>.json)
# Extra bench.py flags: BENCH_FLAGS (default: --no-cpu-baseline --no-roofline)
set -uo pipefail
TAG=$1; ROUNDS=$2; shift 2
O=gpurun_out; mkdir -p $O
FLAGS=${BENCH_FLAGS:---no-cpu-baseline --no-roofline}
for r in $(seq 1 $ROUNDS); do
  i=0
  for v in "$@"; do
    env $v timeout -k 10 200 python3 bench.py $FLAGS > $O/${TAG}_v${i}_r$r.json 2> $O/${TAG}_v${i}_r$r.err || exit $?
    echo "$TAG v$i ($v) round $r: $(python3 -c "import json;print(round(json.load(open('$O/${TAG}_v${i}_r$r.json'))['value']))")"
    i=$((i+1))
  done
done
