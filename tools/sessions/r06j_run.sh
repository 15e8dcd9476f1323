#!/bin/bash
# round 6: re-measure on the final tree what DESIGN.md cited from earlier
# rounds - the single engine's batched dispatch ceiling (zero-cost workers)
# and conv_gemm_big_kernel's stall counters on PoseNet 1024 -> 1024, B = 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
bash tools/ceiling_sweep.sh $O/planner_ceiling_sweep.jsonl || exit 1
echo ceiling done
W=$(mktemp -d /tmp/r06j_XXXX)
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_I8 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES"
n=0
for P in "$P1" "$P2"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$W/stall$n" -o run -- \
    python3 tools/mfma_layer_bench.py --batches 256 --only "posenet 14 1024->1024" --iters 5 > $O/stall$n.log 2>&1 || exit 2
done
python3 tools/pmc_kernels.py --full "$W/stall1" "$W/stall2" > $O/gemm_big_stall.txt || exit 3
rm -rf "$W"
echo done
