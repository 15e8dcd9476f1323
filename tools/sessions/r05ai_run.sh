#!/bin/bash
# round 5: is the chain kernels' depthwise phase bound by the texture
# addresser?  TA / TCP counters on the 56x56 x 144 residual chain (64-pixel
# form) and the 112x112 x 96 stride-2 chain at B = 24, and the standalone
# run-form depthwise layer for comparison
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05ai
mkdir -p $O
W=$(mktemp -d /tmp/prof_XXXX)
P="TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
n=0
for only in 2 1; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$W/c$n" -o run -- \
    python3 tools/chain_bench.py --batch 24 --iters 5 --only $only --px 4 > "$O/chain_$only.log" 2>&1 || exit $n
  python3 tools/pmc_kernels.py "$W/c$n" > "$O/chain_${only}_ta.txt" 2>&1 || exit 5
done
rm -rf "$W"
echo done
