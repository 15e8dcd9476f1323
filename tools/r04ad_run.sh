#!/usr/bin/env bash
# phase-C split A-B on one box: batch-24 breakdown and the 8-stream device
# probe (no I/O), with and without the split candidates, interleaved
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do
  for v in auto nosplit; do
    BAND_HIP_FUSION=$v timeout -k 10 200 python3 tools/mix_breakdown.py --batch 24 > $O/r04ad_breakdown_${v}_r$r.txt 2>&1 || exit 1
  done
done
PROBE_FLAGS=--no-io timeout -k 10 500 bash tools/ab_probe.sh r04ad_probe 24 8 "BAND_HIP_FUSION=auto" "BAND_HIP_FUSION=nosplit" "BAND_HIP_FUSION=auto" "BAND_HIP_FUSION=nosplit" || exit 2
