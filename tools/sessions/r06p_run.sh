#!/bin/bash
# round 6: the single engine's dispatch ceiling at job batch 1 (Band's own
# contract) with 8 / 12 / 96 workers, CPU stand-in work and GPU workers
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06p
mkdir -p $O
: > $O/ceiling_jb1.jsonl
for w in 8 12 96; do
  BANDX_DRIVER_READERS=4 BANDX_DRIVER_LANES=2 timeout -k 10 120 python tools/planner_ceiling.py --workers $w --jobs 200000 >> $O/ceiling_jb1.jsonl 2>/dev/null || exit 1
  BANDX_DRIVER_READERS=4 BANDX_DRIVER_LANES=2 timeout -k 10 120 python tools/planner_ceiling.py --workers $w --jobs 200000 --gpu >> $O/ceiling_jb1.jsonl 2>/dev/null || exit 2
done
echo done
