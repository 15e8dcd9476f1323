#!/usr/bin/env bash
# Interleaved A-B of the closed-loop driver's submitter threads
# (BANDX_DRIVER_LANES) on the default C3 line (no CPU baseline / roofline).
set -uo pipefail
O=gpurun_out; mkdir -p $O
for rep in 1 2; do
  for l in 1 2 3; do
    BANDX_DRIVER_LANES=$l timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline > $O/lanes${l}_r$rep.json 2> $O/lanes${l}_r$rep.err || exit $?
    echo "lanes $l rep $rep done"
  done
done
