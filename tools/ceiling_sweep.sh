#!/bin/bash
# Batched dispatch ceiling (tools/planner_ceiling.py) over the closed-loop
# driver's submitter / reader counts, CPU and GPU workers; one JSON line per
# run into $1 (default gpurun_out/ceiling_sweep.jsonl).
out=${1:-gpurun_out/ceiling_sweep.jsonl}
: > "$out"
run() {
  env "$@" PLANNER_CEILING_SAMPLE=1 timeout -k 10 120 python tools/planner_ceiling.py --workers 8 --job-batch ${CEIL_JB:-32} \
    --jobs 400000 $EXTRA >> "$out" 2>/dev/null || return 1
}
EXTRA="" run BANDX_DRIVER_READERS=2 &&
EXTRA="" run BANDX_DRIVER_READERS=4 BANDX_DRIVER_LANES=2 &&
EXTRA="" run BANDX_DRIVER_READERS=8 BANDX_DRIVER_LANES=4 &&
EXTRA="" run BANDX_DRIVER_READERS=8 BANDX_DRIVER_LANES=8 &&
EXTRA="--gpu" run BANDX_DRIVER_READERS=2 &&
EXTRA="--gpu" run BANDX_DRIVER_READERS=8 BANDX_DRIVER_LANES=4
