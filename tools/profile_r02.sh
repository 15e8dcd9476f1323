#!/usr/bin/env bash
# Round-2 profile set on an MI355X box (outputs in gpurun_out/<tag>_*):
#   0. the default bench line, untraced; the executor's measured kernel /
#      fusion choices go to a tune file that every traced run below replays
#      (tracing distorts the measurements those choices come from);
#   1. the default bench configuration (8 GPU workers, eager launches, job
#      batch <= 24) under rocprofv3 --kernel-trace --stats: per-kernel
#      durations of exactly what bench.py times;
#   2. bench.py --profile-only (the batch-24 passes the roofline line
#      reports) under --kernel-trace --stats;
#   3./4. FETCH_SIZE and WRITE_SIZE passes (separate runs, no other traces)
#      over the same profile-only passes -> tools/pmc_traffic.py;
#   5. FETCH_SIZE over the multi-worker bench itself (8 worker threads).
# Traced runs use eager launches (--no-graph): rocprofv3 7.2 segfaults inside
# hipGraphLaunch in this process; the kernels, their
# grids and the batches are the same as in graph replay.
# usage: tools/profile_r02.sh <tag>
set -euo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p "$O"
export BAND_HIP_TUNE_FILE=$O/${TAG}_tune.txt
rm -f "$BAND_HIP_TUNE_FILE"
timeout -k 10 300 python3 bench.py > "$O/${TAG}_bench_default.json" 2> "$O/${TAG}_bench_default.err"
echo "step 0 done"
KT="rocprofv3 --kernel-trace --stats --output-format csv"
timeout -k 10 400 $KT -d "$O/${TAG}_full" -o run -- python3 bench.py --no-cpu-baseline --no-batch1 --no-graph \
  > "$O/${TAG}_bench_traced.json" 2> "$O/${TAG}_full.err"
echo "step 1 done"
timeout -k 10 200 $KT -d "$O/${TAG}_po" -o run -- python3 bench.py --profile-only --no-graph \
  > "$O/${TAG}_profile_only.json" 2> "$O/${TAG}_po.err"
echo "step 2 done"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/${TAG}_pmcf" -o run -- \
  python3 bench.py --profile-only --no-graph > "$O/${TAG}_pmcf.log" 2> "$O/${TAG}_pmcf.err"
echo "step 3 done"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$O/${TAG}_pmcw" -o run -- \
  python3 bench.py --profile-only --no-graph > "$O/${TAG}_pmcw.log" 2> "$O/${TAG}_pmcw.err"
echo "step 4 done"
python3 tools/pmc_traffic.py "$O/${TAG}_pmcf" "$O/${TAG}_pmcw" "$O/${TAG}_pmc_traffic.json" --batch 24 \
  --config "bench.py --profile-only: C3 mix batch-24 passes" > "$O/${TAG}_pmc_traffic.txt"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/${TAG}_pmcf_full" -o run -- \
  python3 bench.py --no-cpu-baseline --no-batch1 --no-graph --steps 5 --warmup 2 > "$O/${TAG}_pmcf_full.json" 2> "$O/${TAG}_pmcf_full.err"
echo "step 5 done"
python3 tools/pmc_traffic.py "$O/${TAG}_pmcf_full" - "$O/${TAG}_pmc_fetch_full.json" --batch 0 \
  --config "bench.py --no-batch1 --no-graph --steps 5: 8 GPU workers, job batches <= 24 (FETCH_SIZE only)" \
  > "$O/${TAG}_pmc_fetch_full.txt"
# keep the summaries, drop the raw traces (gpurun copies back <= 64 MiB)
for d in full po; do cp "$O/${TAG}_$d/run_kernel_stats.csv" "$O/${TAG}_${d}_kernel_stats.csv"; done
rm -rf "$O/${TAG}_full" "$O/${TAG}_po" "$O/${TAG}_pmcf" "$O/${TAG}_pmcw" "$O/${TAG}_pmcf_full"
echo "profile $TAG done"
