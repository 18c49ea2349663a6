# Round-end verification on the GPU box: full GPU test suite -> e2e CLI checks -> headline bench
# -> rocprofv3 kernel stats. Every GPU step has its own time limit; the chain stops at the first failure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
O=gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_e2e.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
