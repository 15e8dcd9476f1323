#!/bin/bash
# round 5: job coalescer parity tests, then Band's own contract (max_job_batch 1)
# on the C3 mix with coalescing off / on over several worker counts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_coalescer_gpu.py > $O/tests.log 2>&1 || exit 1
run() {  # tag workers [VAR=value ...]
  local tag=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --job-batch 1 --workers-per-gpu $w --steps 10 --warmup 3 \
      --no-cpu-baseline --no-roofline > $O/$tag.json 2> $O/$tag.err || exit 2
}
run w8_off 8 BAND_HIP_COALESCE=0
run w8_on 8 BAND_HIP_COALESCE=16
run w16_on 16 BAND_HIP_COALESCE=16
run w32_on 32 BAND_HIP_COALESCE=16
run w32_l3 32 BAND_HIP_COALESCE=16 BAND_HIP_COALESCE_LANES=3
run w48_b24 48 BAND_HIP_COALESCE=24
echo done
