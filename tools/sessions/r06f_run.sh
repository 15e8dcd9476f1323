#!/bin/bash
# round 6: the GPU suite after the form removals, then the headline defaults A/B, alternating on one box - in flight 384
# (2 x workers x batch, the round-5 default) vs 288 with and without the
# pass-size policy (700 us); job batch 32 at 288 in flight for reference
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
  for v in "384 0 24" "288 0 24" "288 700 24" "256 700 24" "384 700 32"; do
    set -- $v
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --inflight $1 --pass-target-us $2 --job-batch $3 --no-cpu-baseline --no-roofline --no-batch1 \
      > $O/bench_inf$1_pt$2_jb$3_r$r.json 2> $O/bench_inf$1_pt$2_jb$3_r$r.err || exit 1
  done
done
echo done
