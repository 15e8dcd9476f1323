#!/bin/bash
# round 5: coalescer gathering window (BAND_HIP_COALESCE_WAIT_US) over worker
# counts, Band's own contract (max_job_batch 1) on the C3 mix, 1 lane
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_coalescer_gpu.py > $O/tests.log 2>&1 || exit 1
run() {  # tag workers [VAR=value ...]
  local tag=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --job-batch 1 --workers-per-gpu $w --steps 10 --warmup 3 \
      --no-cpu-baseline --no-roofline > $O/$tag.json 2> $O/$tag.err || exit 2
}
for w in 32 48 96; do
  for wt in 0 100 300; do
    run w${w}_wait$wt $w BAND_HIP_COALESCE=24 BAND_HIP_COALESCE_WAIT_US=$wt
  done
done
run w48_wait100_dma 48 BAND_HIP_COALESCE=24 BAND_HIP_COALESCE_WAIT_US=100 BAND_HIP_COALESCE_IO=dma
run w64_wait100 64 BAND_HIP_COALESCE=24 BAND_HIP_COALESCE_WAIT_US=100
echo done
