#!/bin/bash
# round 6: the stage form with loader waves (stage 2) - parity and chain
# times; the headline under the pass-size policy (pass target x in-flight)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chain_gpu.py -k "stage" > $O/tests_stage.log 2>&1 || { tail -30 $O/tests_stage.log; exit 1; }
tail -1 $O/tests_stage.log
F=1w8,1w16,g1w8,g2w8,G1w8,G2w8,G1w4,G2w4,G1w8s2,G2w8s2,G1w8s4,G1w8s8
timeout -k 10 200 python -u tools/chain_bench.py --batch 24 --iters 30 --px $F > $O/chain_b24.txt 2>&1 || exit 4
timeout -k 10 200 python -u tools/chain_bench.py --batch 1 --iters 30 --px $F > $O/chain_b1.txt 2>&1 || exit 5
for pt in 0 500 700; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --inflight 288 --pass-target-us $pt --no-cpu-baseline --no-roofline --no-batch1 \
    > $O/bench_pt${pt}_inf288.json 2> $O/bench_pt${pt}_inf288.err || exit 6
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --pass-target-us 600 --no-cpu-baseline --no-roofline --no-batch1 \
    > $O/bench_pt600_inf384.json 2> $O/bench_pt600_inf384.err || exit 7
echo done
