#!/bin/bash
# round 5, final tree: the C4 (EfficientDet-Lite2, HEFT) and C5 (8-DNN
# Poisson stream, SEL) bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05av
mkdir -p $O
timeout -k 10 300 python3 bench.py --model efficientdet_lite2_int8 --scheduler heterogeneous_earliest_finish_time --job-batch 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 1
timeout -k 10 300 python3 bench.py --model mix_c5 --scheduler shortest_expected_latency --job-batch 1 --rate 4200 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 2
echo done
