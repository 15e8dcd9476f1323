#!/bin/bash
# round 5: why conv_gemm_big_kernel sits at ~18 % of MFMA peak - stall
# counters on the PoseNet 1024x1024 / MobileNetV2 320->1280 layers at B=256
# (micro-benchmark, 5 launches each), plus the tile configurations timed
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
W=$(mktemp -d /tmp/prof_XXXX)
CMD="python3 tools/mfma_layer_bench.py --batches 256 --hint 3 --iters 5 --only 1024->1024"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
n=0
for P in "$P1" "$P2"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$W/stall$n" -o run -- \
    $CMD > "$O/stall$n.log" 2>&1 || exit $n
done
python3 tools/pmc_kernels.py --full "$W/stall1" "$W/stall2" > "$O/stall.txt" || exit 5
for cfg in 1 2 3 4; do
  BH_GEMM_BIG_CFG=$cfg timeout -k 10 200 python3 -u tools/mfma_layer_bench.py --batches 256 --hint 3 --only posenet > $O/cfg$cfg.txt 2>&1 || exit 6
done
rm -rf "$W"
echo done
