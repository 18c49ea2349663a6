# One GPU measurement cycle: GPU tests -> bench -> rocprofv3 kernel stats.
# usage: bash scripts/gpu_cycle.sh TAG [pytest-args...]
TAG=${1:-run}; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TESTS=${@:-tests/test_gpu_probe.py tests/test_gpu_forward.py tests/test_gpu_backward.py tests/test_gpu_compat.py}
timeout -k 10 900 python -m pytest $TESTS -q -m gpu -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log
tail -8 gpurun_out/${TAG}_tests.log
# 0 = pass, 1 = test failures: the GPU is healthy, continue. Anything else (crash/timeout): stop.
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --phases > gpurun_out/${TAG}_bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/${TAG}_bench.log
tail -2 gpurun_out/${TAG}_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1
echo "prof rc=$?"
