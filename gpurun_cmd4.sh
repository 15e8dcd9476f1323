R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python tools/profile_ops.py --iters 50 > gpurun_out/ops4.txt 2>&1 && \
timeout -k 10 120 python tools/profile_ops.py --iters 20 --batch 32 > gpurun_out/ops4_b32.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof4 -o run -- python3 $R/bench.py --steps 1000 --warmup 100 --workers-per-gpu 1 --no-graph --no-cpu-baseline > $R/gpurun_out/prof4.log 2>&1
echo EXIT $?
