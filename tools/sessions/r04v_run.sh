#!/usr/bin/env bash
# tools/graph_copytrace_probe under rocprofv3 --memory-copy-trace, one node mix per
# run; stops at the first fault (the rest of the call runs nothing on the GPU)
export TMPDIR=/tmp
O=gpurun_out
for spec in "$@"; do
  set -- $spec
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/kp_$1_$2 -o run -- \
    ./tools/graph_copytrace_probe $1 1000 20 $2 > $O/r04v_kernarg_$1_$2.log 2>&1
  rc=$?
  echo "graph_copytrace_probe $1 $2 under --memory-copy-trace: rc=$rc" >> $O/r04v_summary.txt
  [ $rc -ne 0 ] && exit 3
done
exit 0
