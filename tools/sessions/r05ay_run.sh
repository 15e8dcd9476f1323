#!/bin/bash
# round 5, HEAD at session end: the driver's round-end sequence - the whole
# GPU suite, smoke(), and the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ay
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo done
