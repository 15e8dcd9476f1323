#!/bin/bash
# round 5: the VALU RGB stem at B = 24 - channel split over grid.y
# (BH_STEM_MIN_WG 512 = default / 2048 / 4096, interleaved x2) and its
# occupancy / stall counters against the GPU's active cycles
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05t
mkdir -p $O
for r in 1 2; do
  for w in 512 2048 4096 9999; do
    BH_STEM_MIN_WG=$w timeout -k 10 120 python3 -u tools/mfma_layer_bench.py --batches 24 --hint 4 --only stem > $O/stem_wg${w}_r$r.txt 2>&1 || exit 1
  done
done
W=$(mktemp -d /tmp/prof_XXXX)
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$W/p1" -o run -- \
  python3 tools/mfma_layer_bench.py --batches 24 --hint 4 --only stem --iters 5 > $O/stem_pmc1.log 2>&1 || exit 2
python3 tools/pmc_kernels.py --full "$W/p1" > $O/stem_pmc.txt 2>&1 || exit 3
python3 -c "import glob,shutil,sys; f=glob.glob(sys.argv[1]+'/**/*counter_collection.csv', recursive=True); f and shutil.copy(f[0], sys.argv[2])" "$W/p1" $O/stem_counters.csv || exit 4
rm -rf "$W"
echo done
