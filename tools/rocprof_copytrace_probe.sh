#!/usr/bin/env bash
# rocprofv3 --memory-copy-trace on the bench under one environment variant
# (verdict item 7): usage tools/rocprof_copytrace_probe.sh <tag> "<ENV=..>" [bench args]
set -uo pipefail
TAG=$1; VAR=$2; shift 2
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
W=$(mktemp -d /tmp/ct_XXXX)
env $VAR timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$W/t" -o run -- \
  python3 bench.py --no-cpu-baseline --no-batch1 --no-roofline --steps 4 --warmup 1 "$@" > "$O/${TAG}.json" 2> "$O/${TAG}.err"
rc=$?
echo "$TAG ($VAR $*): rc=$rc" | tee -a "$O/${TAG}_summary.txt"
grep -h "graphs\|SIGSEGV\|bh_graph_launch\|RunDirect\|TimeSubgraph" "$O/${TAG}.err" | head -5 >> "$O/${TAG}_summary.txt"
cp "$W/t/run_kernel_stats.csv" "$O/${TAG}_kernel_stats.csv" 2>/dev/null
cp "$W/t/run_memory_copy_stats.csv" "$O/${TAG}_copy_stats.csv" 2>/dev/null
rm -rf "$W"
exit $rc
