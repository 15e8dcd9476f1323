#!/usr/bin/env bash
# Reproduces the profiles/ evidence for one round on an MI355X box:
#   1. bench.py (default workload), writing the fused-block tuning decisions
#      to a tune file;
#   2. the same bench command under rocprofv3 --kernel-trace --stats
#      (--no-graph: rocprofv3 crashes inside hipGraphLaunch with kernel
#      tracing; --no-batch1: the stats then hold the headline's batched
#      passes only), replaying the same tuning decisions -> per-kernel
#      durations;
#   3. two PMC passes (FETCH_SIZE, WRITE_SIZE; never combined with
#      sys/runtime traces) -> HBM traffic per launch (tools/pmc_traffic.py).
# usage: tools/profile_bench.sh <tag> [extra bench args]   (outputs in gpurun_out/<tag>_*)
set -euo pipefail
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
O=$R/gpurun_out
mkdir -p "$O"
export BAND_HIP_TUNE_FILE=$O/${TAG}_tune.txt
rm -f "$BAND_HIP_TUNE_FILE"
ARGS="--steps 2000 --warmup 200 --workers-per-gpu 1 $*"
timeout -k 10 300 python3 bench.py $ARGS > "$O/${TAG}_bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${TAG}_trace" -o run -- \
  python3 bench.py $ARGS --no-graph --no-cpu-baseline --no-batch1 > "$O/${TAG}_bench_profiled.json" 2> "$O/${TAG}_trace.err"
# PMC passes: tools/pmc_pass.py replays the bench's batched passes from one
# thread (bench.py itself crashed inside rocprofv3's PMC dispatch hook)
JB=$(python3 -c "import sys; a=sys.argv[1:]; print(a[a.index('--job-batch')+1] if '--job-batch' in a else 24)" $*)
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/${TAG}_pmcf" -o run -- \
  python3 tools/pmc_pass.py --batch $JB > "$O/${TAG}_pmcf.log" 2> "$O/${TAG}_pmcf.err"
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$O/${TAG}_pmcw" -o run -- \
  python3 tools/pmc_pass.py --batch $JB > "$O/${TAG}_pmcw.log" 2> "$O/${TAG}_pmcw.err"
python3 tools/pmc_traffic.py "$O/${TAG}_pmcf" "$O/${TAG}_pmcw" "$O/${TAG}_pmc_traffic.json" > "$O/${TAG}_pmc_traffic.txt"
cp "$O/${TAG}_trace/run_kernel_stats.csv" "$O/${TAG}_kernel_stats.csv"
echo "profile $TAG done"
