#!/bin/bash
# round 5 final tree (LDS-staged stem): the whole GPU suite and smoke(), then
# the profile set (tools/profile_r05.sh r05y: default line, traced bench,
# PMC traffic and stall passes tagged with this kernel tree, final line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
bash tools/profile_r05.sh r05y > $O/profile.log 2>&1 || exit 3
echo done
