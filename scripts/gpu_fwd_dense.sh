# Dense-row controller step: tests (incl. bitwise dense vs 16-slot path), micro A/B, bench
cd $GRAFT_REPO_ROOT
O=gpurun_out/fwd_dense
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fp32.py tests/test_gpu_small.py tests/test_gpu_forward.py tests/test_gpu_backward.py tests/test_gpu_nd.py tests/test_gpu_runtime.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
TAG=fwd_dense PAIRS="fp32:base fp32:nodense bf16:base" bash scripts/gpu_micro_ab.sh
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_fp32.log 2>&1 && tail -1 $O/bench_fp32.log | cut -c1-220
