#!/usr/bin/env bash
# copy-trace check of the padded conv_group_kernel arguments on the bench,
# then the one-node reproducer, padded (clean) and small (faults: last)
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k group --timeout 120 --timeout-method thread > $O/r04u_group_tests.log 2>&1 || exit 1
timeout -k 10 400 bash tools/rocprof_copytrace_probe.sh r04u_grouppad "BAND_HIP_FUSION=auto" || exit 2
for mode in padded small; do
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/kp_$mode -o run -- \
    ./tools/graph_copytrace_probe $mode 1000 20 > $O/r04u_kernarg_$mode.log 2>&1
  rc=$?
  echo "graph_copytrace_probe $mode under --memory-copy-trace: rc=$rc" >> $O/r04u_summary.txt
  grep -h "SIGSEGV\|OK" $O/r04u_kernarg_$mode.log | head -3 >> $O/r04u_summary.txt
  [ $rc -ne 0 ] && exit 3
done
