#!/bin/bash
# round 6: (1) the 16-wave deep chain form (DA 4) and phase-C slices up to 8
# - chain parity, chain_bench at batch 1 / 24, the batch-1 mix; (2) the 2-D
# XCD split of conv_gemm_kernel / conv_mfma_kernel - conv parity, then the
# FETCH_SIZE / WRITE_SIZE passes and the batch-32 mix interleaved against
# libband_hip_head.so (the previous commit's tree)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_chain_gpu.py \
  -k "mnv2 or general or split" > $O/chain_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  > $O/kernel_tests.log 2>&1 || exit 2
echo tests done
F=1w16,1w16d,1w16s2,1w16ds2,1w16ds4,1w16ds8,1w16s8,1w8s8,1w8,1w8d,1d,1s2,G1w8s2,g1w8s8
timeout -k 10 200 python -u tools/chain_bench.py --batch 1 --px $F --iters 200 > $O/chain_b1.txt 2>&1 || exit 3
timeout -k 10 200 python -u tools/chain_bench.py --batch 24 --px $F --iters 50 > $O/chain_b24.txt 2>&1 || exit 4
timeout -k 10 300 python -u tools/mix_breakdown.py --batch 1 --iters 50 > $O/mix_b1.txt 2>&1 || exit 5
echo chain done
W=$(mktemp -d /tmp/r06k_XXXX)
for v in new head new head; do
  if [ $v = head ]; then export BAND_HIP_LIB_VARIANT=head; else unset BAND_HIP_LIB_VARIANT; fi
  timeout -k 10 300 python -u tools/mix_breakdown.py --batch 32 --iters 20 > $O/mix_b32_$v.txt 2>&1 || exit 6
done
for v in new head; do
  if [ $v = head ]; then export BAND_HIP_LIB_VARIANT=head; else unset BAND_HIP_LIB_VARIANT; fi
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$W/f_$v" -o run -- \
    python3 bench.py --profile-only --no-graph > $O/pmcf_$v.log 2>&1 || exit 7
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$W/w_$v" -o run -- \
    python3 bench.py --profile-only --no-graph > $O/pmcw_$v.log 2>&1 || exit 8
  python3 tools/pmc_traffic.py "$W/f_$v" "$W/w_$v" $O/traffic_$v.json --batch 32 --config "xcd A/B $v" \
    > $O/traffic_$v.txt || exit 9
  echo "traffic $v done"
done
unset BAND_HIP_LIB_VARIANT
rm -rf "$W"
echo done
