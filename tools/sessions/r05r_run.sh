#!/bin/bash
# round 5 final tree, part 1: the whole GPU suite, smoke(), and the BASELINE
# configs C2 (with spinning and adaptive waits) / C4 / C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 240 python3 bench.py --model mobilenet_v2_int8 --workers-per-gpu 1 --job-batch 1 --scheduler fixed_worker --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 3
BAND_HIP_SYNC=spin timeout -k 10 240 python3 bench.py --model mobilenet_v2_int8 --workers-per-gpu 1 --job-batch 1 --scheduler fixed_worker --no-cpu-baseline > $O/c2_spin.json 2> $O/c2_spin.err || exit 4
timeout -k 10 300 python3 bench.py --model efficientdet_lite2_int8 --scheduler heterogeneous_earliest_finish_time --job-batch 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 5
timeout -k 10 300 python3 bench.py --model mix_c5 --scheduler shortest_expected_latency --job-batch 1 --rate 4200 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 6
echo done
