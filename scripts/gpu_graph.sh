# Small-config check: eager vs captured graphs, with and without early stopping.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_backward.py tests/test_gpu_compat.py -q -m gpu -p no:cacheprovider > gpurun_out/graph_tests.log 2>&1
rc=$?; tail -3 gpurun_out/graph_tests.log; if [ $rc -gt 1 ]; then exit $rc; fi
for cfg in "--agents 32 --envs 1" "--agents 32 --envs 1 --no_early_stop" "--agents 32 --envs 1 --no_early_stop --graph" "--agents 32 --envs 64 --no_early_stop" "--agents 32 --envs 64 --no_early_stop --graph" ""; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 $cfg > gpurun_out/graph_bench.tmp 2>&1 || { cat gpurun_out/graph_bench.tmp; exit 1; }
  echo "$cfg :: $(tail -1 gpurun_out/graph_bench.tmp | cut -c100-200)" >> gpurun_out/graph_bench.log
  tail -1 gpurun_out/graph_bench.log
done
