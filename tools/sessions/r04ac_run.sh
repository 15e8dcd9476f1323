#!/usr/bin/env bash
# phase-C split: chain parity, per-chain timings (split vs not), batch-24 breakdown
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_chain_gpu.py -x -q --timeout 150 --timeout-method thread > $O/r04ac_chain_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/chain_bench.py --only 4,5,6,7,8,9,10,11 --px 1,1s2,1s3,1w8,1w8s2,2,2s2 --iters 30 > $O/r04ac_chain_bench_b24.txt 2>&1 || exit 2
timeout -k 10 200 python3 tools/chain_bench.py --batch 1 --only 6,7,8,9,10,11 --px 1,1s2,1s3,1w8,1w8s2 --iters 30 > $O/r04ac_chain_bench_b1.txt 2>&1 || exit 3
timeout -k 10 200 python3 tools/mix_breakdown.py --batch 24 > $O/r04ac_breakdown_b24.txt 2>&1 || exit 4
