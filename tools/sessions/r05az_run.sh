#!/bin/bash
# round 5: what bounds the chain kernel's depthwise phase - timing-only
# builds of fused_chain.hip with parts of phase A removed (outputs wrong by
# design; built out of tree from a patched copy, libband_hip_diag{1,2,3}.so):
# 1 = no requantisation, 2 = no MFMA / requantisation, 3 = no tap loads /
# ds_bpermute.  Chain times and per-phase stamps against the default build.
# The variants: patch a copy of band_amd/csrc with tools/sessions/r05az_diag.patch,
# then make -C <copy> ROOT=<repo> BUILD=/tmp/build_diagN OUT=<repo>/band_amd/libband_hip_diagN.so KDEFS=-DBH_DIAG_A=N
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05az
mkdir -p $O
for v in "" diag1 diag2 diag3; do
  BAND_HIP_LIB_VARIANT=$v timeout -k 10 120 python -u tools/chain_bench.py --batch 24 --iters 30 --px 1,2,4,1w8 > $O/chain_${v:-def}.txt 2>&1 || exit 1
  BAND_HIP_LIB_VARIANT=$v timeout -k 10 120 python -u tools/tile_probe.py --batch 24 --raster 2 --only 1,2,4,8 > $O/probe2_${v:-def}.txt 2>&1 || exit 2
  BAND_HIP_LIB_VARIANT=$v timeout -k 10 120 python -u tools/tile_probe.py --batch 24 --raster 1w8 --only 6,8,10 > $O/probe1w8_${v:-def}.txt 2>&1 || exit 3
done
echo done
