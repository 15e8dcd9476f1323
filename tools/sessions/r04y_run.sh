#!/usr/bin/env bash
# final bench lines (PMC traffic now committed for this kernel tree), a C5
# repeat, and job batch 24 vs 32 interleaved
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python3 bench.py > $O/r04y_bench_default.json 2> $O/r04y_bench_default.err || exit 1
timeout -k 10 300 python3 bench.py --model mix_c5 --scheduler shortest_expected_latency --job-batch 1 --rate 4200 --no-cpu-baseline > $O/r04y_c5.json 2> $O/r04y_c5.err || exit 2
for r in 1 2; do
  BANDX_REQUEST_RING_SLOTS=256 timeout -k 10 250 python3 bench.py --no-cpu-baseline --no-batch1 --job-batch 32 > $O/r04y_jb32_r$r.json 2> $O/r04y_jb32_r$r.err || exit 3
  timeout -k 10 250 python3 bench.py --no-cpu-baseline --no-batch1 > $O/r04y_jb24_r$r.json 2> $O/r04y_jb24_r$r.err || exit 4
done
