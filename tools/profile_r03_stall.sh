#!/usr/bin/env bash
# Stall profile of the batch-24 passes (bench.py --profile-only), one
# rocprofv3 --pmc pass per counter group, per kernel instantiation
# (tools/pmc_kernels.py --full).  The tune file of a previous default run
# ($BAND_HIP_TUNE_FILE) makes the passes replay its kernel choices.
# usage: tools/profile_r03_stall.sh <tag>
set -uo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p "$O"
# rocprofv3's pass directories go to a scratch dir (they exceed what a GPU
# call copies back); only the summaries land in gpurun_out
W=$(mktemp -d /tmp/stall_XXXX)
timeout -s KILL 60 rocprofv3 -L > "$O/${TAG}_counters.txt" 2>&1 || true
have() { grep -qw "$1" "$O/${TAG}_counters.txt"; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2=""
for c in SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_I8 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM; do
  if have "$c" && [ "$(echo $P2 | wc -w)" -lt 8 ]; then P2="$P2 $c"; fi
done
echo "pass1: $P1" > "$O/${TAG}_stall_passes.txt"
echo "pass2:$P2" >> "$O/${TAG}_stall_passes.txt"
n=0
for P in "$P1" "$P2"; do
  n=$((n + 1))
  [ -z "$P" ] && continue
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$W/${TAG}_stall$n" -o run -- \
    python3 bench.py --profile-only --no-graph > "$O/${TAG}_stall$n.log" 2>&1
  rc=$?
  echo "pass $n rc=$rc" >> "$O/${TAG}_stall_passes.txt"
  [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_kernels.py --full "$W/${TAG}_stall1" "$W/${TAG}_stall2" > "$O/${TAG}_stall.txt"
rm -rf "$W"
echo "stall $TAG done"
