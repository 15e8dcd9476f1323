#!/bin/bash
# round 5: the MFMA stem with the untransposed epilogue (a lane = 4 pixels of
# one channel: one ChanQ per channel block, quad-transposed dword stores) -
# parity, then against the LDS VALU stem at B = 1 / 24 / 32, interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05z2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem" > $O/tests_stem.log 2>&1 || exit 1
for r in 1 2; do
  for h in 4 5; do
    timeout -k 10 120 python3 -u tools/mfma_layer_bench.py --batches 1,24,32 --hint $h --only stem > $O/stem_h${h}_r$r.txt 2>&1 || exit 2
  done
done
echo done
