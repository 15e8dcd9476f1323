#!/bin/bash
# round 6: what bounds the RGB stem at batch 32 - the two routed forms (LDS
# records / MFMA) under the SQ stall counters, layer_bench only
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06af
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA"
for h in 0 5; do
  echo "hint $h: $(timeout -k 10 120 python tools/layer_bench.py --only stem --batch 32 --iters 50 --dw-hint $h | head -1)" | tee -a $O/time.txt || exit 1
  n=0
  for P in "$P1" "$P2"; do
    n=$((n + 1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/h${h}_p$n" -o run -- \
      python3 tools/layer_bench.py --only stem --batch 32 --iters 5 --dw-hint $h > $O/h${h}_p$n.log 2>&1 || { tail -5 $O/h${h}_p$n.log; exit 1; }
  done
  python3 tools/pmc_kernels.py --full $O/h${h}_p1 $O/h${h}_p2 > $O/h${h}_stall.txt || exit 1
done
echo done
