#!/bin/bash
# round 5: stem on MFMA + phase-C split parity; then interleaved same-box
# A/Bs: the phase-C split forms (BAND_HIP_FUSION=nosplit vs default) on the
# batch-24 mix kernel sum and the C3 headline; the completion poller
# (BAND_HIP_SYNC=poller) vs spinning waits; Band's own contract with it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_chain_gpu.py -k "stem or split" > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_coalescer_gpu.py > $O/tests_coalescer.log 2>&1 || exit 1
for r in 1 2; do
  BAND_HIP_FUSION=nosplit timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 > $O/breakdown_nosplit_r$r.txt 2>&1 || exit 2
  timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 > $O/breakdown_split_r$r.txt 2>&1 || exit 3
done
timeout -k 10 300 python -u tools/mix_breakdown.py --batch 1 --models mobilenet_v2 --top 30 > $O/breakdown_mnv2_b1.txt 2>&1 || exit 9
B="--no-cpu-baseline --no-roofline --no-batch1 --no-single-engine"
for r in 1 2; do
  BAND_HIP_FUSION=nosplit timeout -k 10 300 python bench.py $B > $O/bench_nosplit_r$r.json 2> $O/bench_nosplit_r$r.err || exit 4
  timeout -k 10 300 python bench.py $B > $O/bench_split_r$r.json 2> $O/bench_split_r$r.err || exit 5
done
for r in 1 2; do
  BAND_HIP_SYNC=poller timeout -k 10 300 python bench.py $B > $O/bench_poller_r$r.json 2> $O/bench_poller_r$r.err || exit 6
  timeout -k 10 300 python bench.py $B > $O/bench_spin_r$r.json 2> $O/bench_spin_r$r.err || exit 7
done
BAND_HIP_SYNC=poller timeout -k 10 300 python bench.py --job-batch 1 --workers-per-gpu 48 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/band1_poller.json 2> $O/band1_poller.err || exit 8
echo done
