#!/bin/bash
# round 6 final tree (MFMA stem at every batch, multi-row resize, latency
# point 24 / 450 / 200), part 1: the GPU suite, smoke(), BASELINE configs
# C2 / C4 / C5, the mix breakdowns at batch 32 and 1, two default lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06am
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
tail -1 $O/smoke.log
timeout -k 10 240 python3 bench.py --model mobilenet_v2_int8 --workers-per-gpu 1 --job-batch 1 --scheduler fixed_worker --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 3
timeout -k 10 300 python3 bench.py --model efficientdet_lite2_int8 --scheduler heterogeneous_earliest_finish_time --job-batch 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 4
timeout -k 10 300 python3 bench.py --model mix_c5 --scheduler shortest_expected_latency --job-batch 1 --rate 4200 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 5
echo configs done
timeout -k 10 400 python -u tools/mix_breakdown.py --batch 32 --top 400 > $O/breakdown_b32.txt 2>&1 || exit 6
timeout -k 10 400 python -u tools/mix_breakdown.py --batch 1 --top 400 > $O/breakdown_b1.txt 2>&1 || exit 7
echo breakdowns done
for r in 1 2; do
  timeout -k 10 420 python -u bench.py > $O/bench_default_r$r.json 2> $O/bench_default_r$r.err || exit 8
done
echo done
