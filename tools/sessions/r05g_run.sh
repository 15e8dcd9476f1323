#!/bin/bash
# round 5, part 2: interleaved same-box A/Bs on the final kernel tree
#  - batch-24 mix kernel sum (tools/mix_breakdown.py): the chain tuner with
#    every form (default) vs without the phase-C split forms (nosplit) vs
#    without the VALU depthwise forms (novalu)
#  - the C3 headline: default vs round 4's chain form set (nosplit + novalu
#    = BAND_HIP_FUSION=r4forms) vs the completion poller (BAND_HIP_SYNC=poller)
#  - Band's own contract (max_job_batch 1, 48 workers) with the poller
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05g
mkdir -p $O
for r in 1 2; do
  for arm in nosplit novalu default; do
    if [ $arm = default ]; then unset BAND_HIP_FUSION; else export BAND_HIP_FUSION=$arm; fi
    timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 > $O/breakdown_${arm}_r$r.txt 2>&1 || exit 2
  done
done
unset BAND_HIP_FUSION
B="--no-cpu-baseline --no-roofline --no-batch1 --no-single-engine"
for r in 1 2; do
  BAND_HIP_FUSION=r4forms timeout -k 10 300 python bench.py $B > $O/bench_r4forms_r$r.json 2> $O/bench_r4forms_r$r.err || exit 4
  timeout -k 10 300 python bench.py $B > $O/bench_default_r$r.json 2> $O/bench_default_r$r.err || exit 5
  BAND_HIP_SYNC=poller timeout -k 10 300 python bench.py $B > $O/bench_poller_r$r.json 2> $O/bench_poller_r$r.err || exit 6
done
BAND_HIP_SYNC=poller timeout -k 10 300 python bench.py --job-batch 1 --workers-per-gpu 48 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/band1_poller.json 2> $O/band1_poller.err || exit 8
echo done
