#!/usr/bin/env bash
# The profile set on an MI355X box (outputs in gpurun_out/<tag>_*;
# rocprofv3's own directories stay in a scratch dir on the box):
#   0. the default bench line, untraced; its measured kernel / fusion
#      choices go to a tune file every later run replays (commit it as
#      profiles/<tag>_tune.tsv beside the PMC traffic file: a default
#      bench.py on the same kernel tree replays it, so its roofline traffic
#      describes the same launches);
#   1. the bench itself (direct ring I/O, 8 GPU workers) WITH its roofline
#      stage under rocprofv3 --kernel-trace --stats, eager launches
#      (--no-graph: rocprofv3 7.2 faults inside hipGraphLaunch after enough
#      graph launches, tools/graph_copytrace_probe.hip)
#      -> kernel stats and tools/timeline_summary.py;
#   2. bench.py --profile-only (the batch-24 passes the roofline line
#      reports) under --kernel-trace --stats;
#   3./4. FETCH_SIZE and WRITE_SIZE passes (separate runs, no other traces)
#      over the same profile-only passes -> tools/pmc_traffic.py, tagged with
#      the kernel tree (bench.py reports `traffic` only for that tree);
#   5./6. the stall counters (two SQ passes) -> tools/pmc_kernels.py --full;
#   7. the default bench line again, now with the PMC traffic in place.
# Profile-only passes use eager launches (--no-graph): same kernels, grids
# and batches as the graph replay.
# usage: tools/profile_set.sh <tag>
set -uo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p "$O"
W=$(mktemp -d /tmp/prof_XXXX)
export BAND_HIP_TUNE_FILE=$O/${TAG}_tune.txt
rm -f "$BAND_HIP_TUNE_FILE"
step() { echo "$(date +%T) $*"; }
timeout -k 10 500 python3 bench.py > "$O/${TAG}_bench_default.json" 2> "$O/${TAG}_bench_default.err" || exit $?
step "0 default line done"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$W/${TAG}_full" -o run -- \
  python3 bench.py --no-cpu-baseline --no-batch1 --no-graph --steps 8 --warmup 2 \
  > "$O/${TAG}_bench_traced.json" 2> "$O/${TAG}_full.err" || exit $?
python3 tools/timeline_summary.py "$W/${TAG}_full/run_kernel_trace.csv" > "$O/${TAG}_timeline.txt" || exit $?
step "1 traced graph-replay bench done"
KT="rocprofv3 --kernel-trace --stats --output-format csv"
timeout -k 10 300 $KT -d "$W/${TAG}_po" -o run -- python3 bench.py --profile-only --no-graph \
  > "$O/${TAG}_profile_only.json" 2> "$O/${TAG}_po.err" || exit $?
step "2 profile-only trace done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$W/${TAG}_pmcf" -o run -- \
  python3 bench.py --profile-only --no-graph > "$O/${TAG}_pmcf.log" 2> "$O/${TAG}_pmcf.err" || exit $?
step "3 FETCH_SIZE done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$W/${TAG}_pmcw" -o run -- \
  python3 bench.py --profile-only --no-graph > "$O/${TAG}_pmcw.log" 2> "$O/${TAG}_pmcw.err" || exit $?
step "4 WRITE_SIZE done"
# the batch the profile-only passes ran at (bench.py's default job batch)
PB=$(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['pass_batch'])" \
  "$O/${TAG}_profile_only.json") || exit $?
python3 tools/pmc_traffic.py "$W/${TAG}_pmcf" "$W/${TAG}_pmcw" "$O/${TAG}_pmc_traffic.json" --batch "$PB" \
  --config "bench.py --profile-only: C3 mix batch-$PB passes" > "$O/${TAG}_pmc_traffic.txt" || exit $?
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_I8 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"
n=0
for P in "$P1" "$P2"; do
  n=$((n + 1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$W/${TAG}_stall$n" -o run -- \
    python3 bench.py --profile-only --no-graph > "$O/${TAG}_stall$n.log" 2>&1 || exit $?
  step "$((n + 4)) stall pass $n done"
done
python3 tools/pmc_kernels.py --full "$W/${TAG}_stall1" "$W/${TAG}_stall2" > "$O/${TAG}_stall.txt" || exit $?
for d in full po; do cp "$W/${TAG}_$d/run_kernel_stats.csv" "$O/${TAG}_${d}_kernel_stats.csv"; done
rm -rf "$W"
# the traffic file must sit under profiles/ for bench.py to report it
cp "$O/${TAG}_pmc_traffic.json" profiles/ || exit $?
timeout -k 10 500 python3 bench.py > "$O/${TAG}_bench_final.json" 2> "$O/${TAG}_bench_final.err" || exit $?
step "7 final default line done"
echo "profile $TAG done"
