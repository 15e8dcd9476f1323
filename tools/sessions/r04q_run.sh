#!/usr/bin/env bash
# stall counters of the batch-24 passes, then the traced bench with its
# roofline stage (verdict item 7)
export TMPDIR=/tmp
timeout -k 10 560 bash tools/profile_r03_stall.sh r04q || exit 3
timeout -k 10 560 bash tools/trace_roofline.sh r04q || exit 4
