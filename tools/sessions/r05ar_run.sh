#!/bin/bash
# round 5: job-batch variant graphs captured at prepare time
# (BAND_HIP_PRECAPTURE, default) against the lazy second-run capture - the
# batched-pass / engine / coalescer GPU tests, then default bench lines
# alternating the two, each with its wall time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ar
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_job_batch_gpu.py tests/test_engine_gpu.py tests/test_coalescer_gpu.py > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in 1 0; do
    s=$(date +%s)
    BAND_HIP_PRECAPTURE=$v timeout -k 10 500 python3 bench.py > $O/bench_pc${v}_r$r.json 2> $O/bench_pc${v}_r$r.err || exit 2
    echo "pc$v r$r wall $(( $(date +%s) - s )) s" >> $O/walls.txt
  done
done
echo done
