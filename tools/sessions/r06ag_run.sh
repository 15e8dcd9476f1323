#!/bin/bash
# round 6: the MFMA stem at the bench's batches - register allocation for 8
# waves per SIMD (WPE 6 launch bound: 64 VGPRs at 4 blocks per wave instead
# of 96) and blocks per wave, against the routed LDS form; parity under the
# new allocation first; two rounds interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06ag
mkdir -p $O
BH_STEM_MFMA_WPE=6 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "conv_stem or first_layer" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for b in 32 24 16; do
    for v in "h0" "h5" "h5 BH_STEM_MFMA_WPE=6" "h5 BH_STEM_MFMA_PB=2"; do
      h=${v%% *}; e=""; [ "$v" != "$h" ] && e=${v#* }
      echo "round $r batch $b $v: $(env $e timeout -k 10 120 python tools/layer_bench.py --only stem --batch $b --iters 50 --dw-hint ${h#h} | head -1)" \
        | tee -a $O/stem.txt || exit 1
    done
  done
done
echo done
