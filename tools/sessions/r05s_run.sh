#!/bin/bash
# round 5: the chain kernel's VALU depthwise phase against the MFMA tile -
# per-chain times at B = 24 and the stall counters of both forms; then the
# headline with 8 / 12 / 16 GPU workers now that waits sleep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 300 python3 -u tools/chain_bench.py --batch 24 --px "4,4v,2,2v,1,1v,1w16,1w16v" > $O/chain_valu_b24.txt 2>&1 || exit 1
W=$(mktemp -d /tmp/prof_XXXX)
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM"
for form in 4 4v; do
  n=0
  for P in "$P1" "$P2"; do
    n=$((n + 1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$W/${form}_$n" -o run -- \
      python3 tools/chain_bench.py --batch 24 --iters 5 --only 2,6 --px $form > "$O/stall_${form}_$n.log" 2>&1 || exit 2
  done
  python3 tools/pmc_kernels.py --full "$W/${form}_1" "$W/${form}_2" > "$O/chain_stall_$form.txt" || exit 3
done
rm -rf "$W"
B="--no-cpu-baseline --no-roofline --no-batch1 --no-single-engine"
for w in 8 12 16; do
  timeout -k 10 300 python bench.py $B --workers-per-gpu $w > $O/bench_w$w.json 2> $O/bench_w$w.err || exit 4
done
echo done
