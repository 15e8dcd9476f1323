#!/usr/bin/env bash
# BASELINE configs C2 / C4 / C5 on the current tree (outputs gpurun_out/<tag>_c*.json)
set -uo pipefail
TAG=${1:?tag}
O=gpurun_out; mkdir -p $O
timeout -k 10 240 python3 bench.py --model mobilenet_v2_int8 --workers-per-gpu 1 --job-batch 1 --scheduler fixed_worker --no-cpu-baseline > $O/${TAG}_c2.json 2> $O/${TAG}_c2.err || exit $?
echo c2 done
timeout -k 10 300 python3 bench.py --model efficientdet_lite2_int8 --scheduler heterogeneous_earliest_finish_time --job-batch 1 --no-cpu-baseline > $O/${TAG}_c4.json 2> $O/${TAG}_c4.err || exit $?
echo c4 done
timeout -k 10 300 python3 bench.py --model mix_c5 --scheduler shortest_expected_latency --job-batch 1 --rate 4200 --no-cpu-baseline > $O/${TAG}_c5.json 2> $O/${TAG}_c5.err || exit $?
echo c5 done
