# Quick GPU iteration: selected GPU tests -> per-step micro-benchmark -> bench (-> optional rocprof).
# usage: bash scripts/gpu_quick.sh TAG [prof] -- pytest-args...
TAG=${1:-q}; shift
PROF=0; if [ "$1" = "prof" ]; then PROF=1; shift; fi
[ "$1" = "--" ] && shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 300 python scripts/micro_step.py --tag $TAG > gpurun_out/${TAG}_micro.log 2>&1 || { tail -5 gpurun_out/${TAG}_micro.log; exit 1; }
tail -1 gpurun_out/${TAG}_micro.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --phases > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-200
if [ $PROF = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1
  echo "prof rc=$?"
fi
