#!/usr/bin/env bash
# Interleaved A-B of bench.py variants given as "ENV=.. -- ARGS" strings.
# Usage: tools/ab_args_env.sh TAG ROUNDS "VAR=x -- --job-batch 32" "-- --inflight 512" ...
set -uo pipefail
TAG=$1; ROUNDS=$2; shift 2
O=gpurun_out; mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  i=0
  for v in "$@"; do
    envs=${v%%--*}; args=${v#*--}
    env $envs timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline $args > $O/${TAG}_v${i}_r$r.json 2> $O/${TAG}_v${i}_r$r.err || exit $?
    echo "$TAG v$i ($v) round $r: $(python3 -c "import json;d=json.load(open('$O/${TAG}_v${i}_r$r.json'));h=d['host_threads_timed'];print(round(d['value']), round(d['p99_job_latency_ms'],2), h['worker_phases']['passes'])")"
    i=$((i+1))
  done
done
