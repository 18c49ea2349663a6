# Kernel-level profile of the smallest config (32 agents x 1 env), eager and graph mode.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_small -o run --output-format csv -- python3 $R/bench.py --agents 32 --envs 1 --steps 5 --warmup 2 > $R/gpurun_out/prof_small.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_small_g -o run --output-format csv -- python3 $R/bench.py --agents 32 --envs 1 --steps 5 --warmup 2 --graph > $R/gpurun_out/prof_small_g.log 2>&1
echo "rc=$?"
