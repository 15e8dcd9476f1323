set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_config_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/xcd_tests.log 2>&1 || exit $?
echo tests done
for mode in 1 d; do
  if [ $mode = d ]; then unset BH_CONV_XCD; else export BH_CONV_XCD=$mode; fi
  timeout -k 10 200 python tools/mix_breakdown.py --batch 24 --top 200 > $O/xcd${mode}_mix.txt 2>&1 || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/xcd${mode}_$c -o run -- python3 bench.py --profile-only --no-graph > $O/xcd${mode}_$c.log 2>&1 || exit $?
  done
  python3 tools/pmc_traffic.py $O/xcd${mode}_FETCH_SIZE $O/xcd${mode}_WRITE_SIZE $O/xcd${mode}_traffic.json --batch 24 --config ab > $O/xcd${mode}_traffic.txt || exit $?
  rm -rf $O/xcd${mode}_FETCH_SIZE $O/xcd${mode}_WRITE_SIZE
  echo mode $mode done
done
