#!/bin/bash
# round 5, committed final tree (kernels r05i, graphs captured at prepare
# time): the whole GPU suite, smoke(), C2 and two default bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05as
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 240 python3 bench.py --model mobilenet_v2_int8 --workers-per-gpu 1 --job-batch 1 --scheduler fixed_worker --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 3
for r in 1 2; do
  timeout -k 10 500 python3 bench.py > $O/bench_r$r.json 2> $O/bench_r$r.err || exit 4
done
echo done
