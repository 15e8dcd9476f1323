#!/usr/bin/env bash
# The bench line WITH its roofline stage (TimeSubgraph / ProfileSubgraph
# replays) under rocprofv3: kernel trace alone, then kernel + memory-copy
# trace (the round-3 SIGSEGV configuration, profiles/r03n_traced_bench_crash.txt).
# Each run's exit status and the tail of its stderr go to
# gpurun_out/<tag>_trace_roofline.txt; kernel stats are kept per run.
# usage: tools/trace_roofline.sh <tag>
set -uo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p "$O"
S="$O/${TAG}_trace_roofline.txt"
: > "$S"
W=$(mktemp -d /tmp/trace_XXXX)  # trace directories stay on the box
n=0
for TR in "--kernel-trace" "--kernel-trace --memory-copy-trace"; do
  n=$((n + 1))
  timeout -k 10 400 rocprofv3 $TR --stats --output-format csv -d "$W/${TAG}_tr$n" -o run -- \
    python3 bench.py --no-cpu-baseline --no-batch1 --steps 8 --warmup 2 \
    > "$O/${TAG}_tr$n.json" 2> "$O/${TAG}_tr$n.err"
  rc=$?
  echo "run $n ($TR, roofline stage on): rc=$rc" >> "$S"
  tail -5 "$O/${TAG}_tr$n.err" >> "$S"
  cp "$W/${TAG}_tr$n/run_kernel_stats.csv" "$O/${TAG}_tr${n}_kernel_stats.csv" 2>/dev/null
  rm -rf "$W/${TAG}_tr$n"
  [ $rc -ne 0 ] && exit $rc
done
echo "trace_roofline $TAG done" >> "$S"
