export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04o_gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/mix_breakdown.py --batch 24 > gpurun_out/r04o_breakdown_b24.txt 2>&1 || exit 2
BAND_HIP_LIB_VARIANT=q0 timeout -k 10 200 python tools/mix_breakdown.py --batch 24 > gpurun_out/r04o_breakdown_b24_q0.txt 2>&1 || exit 3
timeout -k 10 700 tools/ab_probe.sh r04o_probe 24 8 "BAND_HIP_LIB_VARIANT=" "BAND_HIP_LIB_VARIANT=q0" "BAND_HIP_LIB_VARIANT=" "BAND_HIP_LIB_VARIANT=q0" || exit 4
timeout -k 10 400 tools/profile_r03_stall.sh r04o || exit 5
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r04o_jb24_r$r.json 2> gpurun_out/r04o_jb24_r$r.err || exit 6
  BANDX_REQUEST_RING_SLOTS=256 timeout -k 10 300 python3 bench.py --no-cpu-baseline --job-batch 32 > gpurun_out/r04o_jb32_r$r.json 2> gpurun_out/r04o_jb32_r$r.err || exit 7
done
