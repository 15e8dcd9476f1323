set -uo pipefail
O=gpurun_out
for r in 1 2; do
for L in 1 4 2; do
  BANDX_DRIVER_LANES=$L timeout -k 10 200 python bench.py --no-cpu-baseline > $O/r04c_lanes${L}_r$r.json 2> $O/r04c_lanes${L}_r$r.err || exit $?
  echo "lanes $L run $r done"
done
done
