#!/bin/bash
# round 5: coalescer I/O modes (dma / copy) and lanes over worker counts,
# Band's own contract (max_job_batch 1) on the C3 mix
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_coalescer_gpu.py > $O/tests.log 2>&1 || exit 1
run() {  # tag workers [VAR=value ...]
  local tag=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --job-batch 1 --workers-per-gpu $w --steps 10 --warmup 3 \
      --no-cpu-baseline --no-roofline > $O/$tag.json 2> $O/$tag.err || exit 2
}
for w in 48 96; do
  for l in 1 2; do
    for io in dma copy; do
      run w${w}_l${l}_$io $w BAND_HIP_COALESCE=24 BAND_HIP_COALESCE_LANES=$l BAND_HIP_COALESCE_IO=$io
    done
  done
done
run w64_l2_dma 64 BAND_HIP_COALESCE=24 BAND_HIP_COALESCE_LANES=2 BAND_HIP_COALESCE_IO=dma
echo done
