#!/bin/bash
# round 6: is C5's intermittent p99 tail (r06am 15.5 ms, r06ao 21.7 ms in
# one of three) new with this round's stem / resize routing?  C5 on the
# final library against the r06w library (libband_hip_old.so, built from
# commit dc643b1), interleaved, three rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06ap
mkdir -p $O
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export BAND_HIP_LIB_VARIANT=old; else unset BAND_HIP_LIB_VARIANT; fi
    timeout -k 10 300 python3 bench.py --model mix_c5 --scheduler shortest_expected_latency --job-batch 1 --rate 4200 --no-cpu-baseline > $O/c5_${v}_r$r.json 2> $O/c5_${v}_r$r.err || exit 1
    python3 -c "import json;d=json.load(open('$O/c5_${v}_r$r.json'));print('c5 $v round $r', round(d['value']), round(d['p50_job_latency_ms'],2), round(d['p99_job_latency_ms'],2))"
  done
done
echo done
