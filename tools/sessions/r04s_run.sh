#!/usr/bin/env bash
# round-4 box session: batched dispatch ceiling sweep, then the bank-conflict
# A/B and chain timings and the copy-trace probe (tools/sessions/r04r_run.sh)
export TMPDIR=/tmp
timeout -k 10 500 bash tools/ceiling_sweep.sh gpurun_out/r04s_ceiling.jsonl || exit 1
timeout -k 10 650 bash tools/sessions/r04r_run.sh || exit $((10 + $?))
