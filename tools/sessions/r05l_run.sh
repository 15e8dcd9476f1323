#!/bin/bash
# round 5: same-box A/B of the batch-24 mix kernel sum, the round-4 tree
# (abtree/r04: its own python + library, built from commit aa4cf12) against
# this tree; the RGB stem's VALU and MFMA forms at B = 24; stall counters of
# the default big-GEMM tile on PoseNet 1024 -> 1024 at B = 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
for r in 1 2; do
  (cd abtree/r04 && timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24) > $O/breakdown_r04tree_r$r.txt 2>&1 || exit 1
  timeout -k 10 300 python -u tools/mix_breakdown.py --batch 24 > $O/breakdown_now_r$r.txt 2>&1 || exit 2
done
for r in 1 2 3; do
  for h in 4 5; do
    timeout -k 10 120 python3 -u tools/mfma_layer_bench.py --batches 24,32 --hint $h --only stem > $O/stem_h${h}_r$r.txt 2>&1 || exit 3
  done
done
W=$(mktemp -d /tmp/prof_XXXX)
CMD="python3 tools/mfma_layer_bench.py --batches 256 --iters 5 --only 1024->1024"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
n=0
for P in "$P1" "$P2"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$W/stall$n" -o run -- \
    $CMD > "$O/stall$n.log" 2>&1 || exit $((3 + n))
done
python3 tools/pmc_kernels.py --full "$W/stall1" "$W/stall2" > "$O/gemm_big_stall.txt" || exit 6
rm -rf "$W"
echo done
