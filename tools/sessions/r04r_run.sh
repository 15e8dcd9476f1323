#!/usr/bin/env bash
# LDS bank conflicts of single chain launches, round-start kernels
# (libband_hip_old.so, built from the round-3 final chain sources at
# 0909fc9) vs this tree; chain timings; then the copy-trace probe (last: a
# tool SIGSEGV ends the GPU work of the call)
export TMPDIR=/tmp
O=gpurun_out
W=$(mktemp -d /tmp/r04r_XXXX)
for spec in "0 t" "2 4" "6 1"; do
  set -- $spec
  for V in old new; do
    VAR=""; [ $V = old ] && VAR=old
    BAND_HIP_LIB_VARIANT=$VAR timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES \
      --kernel-trace --output-format csv -d "$W/c$1_$V" -o run -- python3 tools/chain_bench.py --only $1 --px $2 --iters 20 \
      > "$O/r04r_conf_c$1_$V.log" 2>&1 || exit 1
    python3 tools/pmc_kernels.py --full "$W/c$1_$V" > "$O/r04r_conf_c$1_$V.txt" 2>&1 || exit 1
  done
done
for V in old new; do
  VAR=""; [ $V = old ] && VAR=old
  BAND_HIP_LIB_VARIANT=$VAR timeout -k 10 200 python3 tools/chain_bench.py --px 4,2,1,1w8,t,t3,t4 --iters 30 > "$O/r04r_chain_bench_$V.txt" 2>&1 || exit 2
done
rm -rf "$W"
timeout -k 10 400 bash tools/rocprof_copytrace_probe.sh r04r_step25 BAND_HIP_BATCH_STEP=25 || exit 3
