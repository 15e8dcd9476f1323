#!/usr/bin/env bash
# Device-side A-B (no Band engine, no host request path): the C3 mix's
# batched graphs replayed from S streams (tools/concurrency_probe.py) under
# environment variants.  Usage: tools/ab_probe.sh TAG BATCH STREAMS "ENV A" "ENV B" ...
set -uo pipefail
TAG=$1; B=$2; S=$3; shift 3
O=gpurun_out; mkdir -p $O
i=0
for v in "$@"; do
  env $v timeout -k 10 300 python3 tools/concurrency_probe.py --model mix --batch $B --streams $S --iters 60 ${PROBE_FLAGS:-} > $O/${TAG}_v$i.txt 2>&1 || exit $?
  echo "$TAG v$i ($v): $(grep -E 'inf/s|inferences' $O/${TAG}_v$i.txt | tail -2 | tr '\n' ' ')"
  i=$((i+1))
done
