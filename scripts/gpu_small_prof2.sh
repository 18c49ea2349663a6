# Kernel trace + stats of config #2 (32 agents x 1 env, fp32) and the 8-env strong-scaling slice.
# Output: gpurun_out/${TAG:-smallprof}
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-smallprof}
mkdir -p $O
timeout -k 10 200 python bench.py --agents 32 --envs 1 --steps 30 --warmup 5 --phases > $O/cfg2.log 2>&1 || { tail -5 $O/cfg2.log; exit 1; }
tail -1 $O/cfg2.log | cut -c1-200
timeout -k 10 200 python bench.py --envs 8 --steps 10 --warmup 3 --phases > $O/slice8.log 2>&1 || { tail -5 $O/slice8.log; exit 1; }
tail -1 $O/slice8.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --agents 32 --envs 1 --steps 10 --warmup 3 > $O/prof2.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --envs 8 --steps 5 --warmup 2 > $O/prof8.log 2>&1 || exit 1
