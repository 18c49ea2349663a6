# Small-config (BASELINE #2: 32 agents, 1 env) phase breakdown + kernel trace.
# usage: bash scripts/gpu_small_prof.sh TAG
TAG=${1:-cfg2}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 120 python bench.py --agents 32 --envs 1 --steps 20 --warmup 3 --phases > gpurun_out/${TAG}_phases.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o run --output-format csv -- python3 $R/bench.py --agents 32 --envs 1 --steps 5 --warmup 2 > $R/gpurun_out/${TAG}_prof.log 2>&1
echo "prof rc=$?"
