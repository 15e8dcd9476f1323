#!/usr/bin/env bash
# final kernel tree: every GPU test, smoke, single-chain LDS conflicts
# (chain 0 = 112x112 x 32, tile form), then the full profile set
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04z_gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04z_smoke.log 2>&1 || exit 2
W=$(mktemp -d /tmp/r04z_XXXX)
for spec in "0 t" "2 4"; do
  set -- $spec
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES \
    --kernel-trace --output-format csv -d "$W/c$1" -o run -- python3 tools/chain_bench.py --only $1 --px $2 --iters 20 \
    > "$O/r04z_conf_c$1.log" 2>&1 || exit 3
  python3 tools/pmc_kernels.py --full "$W/c$1" > "$O/r04z_conf_c$1.txt" 2>&1 || exit 3
done
rm -rf "$W"
timeout -k 10 700 bash tools/profile_r04.sh r04z || exit 4
