#!/bin/bash
# round 5: the rest of the chain-kernel component study (timing-only builds
# from tools/sessions/r05az_diag.patch, outputs wrong by design): 4 = no
# second 1x1 (phase C), 5 = no first 1x1 (phase B), 6 = no HBM stores;
# chain times against the default build, twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ba
mkdir -p $O
for r in 1 2; do
  for v in "" diag4 diag5 diag6; do
    BAND_HIP_LIB_VARIANT=$v timeout -k 10 120 python -u tools/chain_bench.py --batch 24 --iters 30 --px 1,2,4,1w8 > $O/chain_${v:-def}_r$r.txt 2>&1 || exit 1
  done
done
echo done
