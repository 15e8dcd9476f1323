#!/usr/bin/env bash
# after the round_robin compaction: engine / job-batch GPU tests, the
# batched dispatch ceiling sweep, and one default bench line
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04af_gpu_tests.log 2>&1 || exit 1
timeout -k 10 500 bash tools/ceiling_sweep.sh $O/r04af_ceiling.jsonl || exit 2
timeout -k 10 300 python3 bench.py > $O/r04af_bench.json 2> $O/r04af_bench.err || exit 3
