#!/usr/bin/env bash
# round-4 checkpoint on a box: chain parity, batch-24 breakdown, stall
# counters, the traced bench with its roofline stage
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_chain_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r04p_chain_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/mix_breakdown.py --batch 24 > gpurun_out/r04p_breakdown_b24.txt 2>&1 || exit 2
timeout -k 10 500 tools/profile_r03_stall.sh r04p || exit 3
timeout -k 10 400 tools/trace_roofline.sh r04p || exit 4
