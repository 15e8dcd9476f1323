R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rows_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/rows_tests.log; exit 1; }
tail -1 gpurun_out/rows_tests.log
BH_CONV_ROWS_MIN_M=0 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rows_all_tests.log 2>&1 || { echo "forced-xs tests failed"; tail -40 gpurun_out/rows_all_tests.log; exit 1; }
tail -1 gpurun_out/rows_all_tests.log
BH_CONV_ROWS_MIN_M=0 timeout -k 10 120 python -u tools/layer_bench.py --batch 64 --only conv > gpurun_out/lb_conv_xs.txt 2>&1
BH_CONV_ROWS_MIN_M=0 BH_CONV_XS=0 timeout -k 10 120 python -u tools/layer_bench.py --batch 64 --only conv > gpurun_out/lb_conv_rows.txt 2>&1
BH_CONV_ROWS_MIN_M=0 timeout -k 10 120 python -u tools/layer_bench.py --batch 1 --only conv > gpurun_out/lb_conv_xs_b1.txt 2>&1
BH_CONV_ROWS_MIN_M=1000000000 timeout -k 10 120 python -u tools/layer_bench.py --batch 1 --only conv > gpurun_out/lb_conv_old_b1.txt 2>&1
echo done
