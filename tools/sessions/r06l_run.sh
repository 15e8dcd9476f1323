#!/bin/bash
# round 6: first GPU run of the image-resident chain sequence - parity, then
# timing against the chains launched one by one at batch 1 / 2 / 4 / 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_chain_seq_gpu.py \
  > $O/seq_tests.log 2>&1 || exit 1
for b in 1 2 4 8; do
  timeout -k 10 120 python -u tools/seq_bench.py --batch $b > $O/seq_bench_b$b.txt 2>&1 || exit 2
done
echo done
