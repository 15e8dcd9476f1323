#!/usr/bin/env bash
# final-tree checks: every GPU test, smoke, then one copy-trace bisection
# step (last: a tool SIGSEGV ends the GPU work of the call)
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04t_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04t_smoke.log 2>&1 || exit 2
timeout -k 10 400 bash tools/rocprof_copytrace_probe.sh r04t_nogroup BAND_HIP_FUSION=nogroup || exit 3
