# Per-group agent base (no per-tile division by N): tests, then interleaved micro A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out/divs
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fp32.py tests/test_gpu_backward.py tests/test_gpu_small.py tests/test_gpu_nd.py tests/test_gpu_runtime.py tests/test_gpu_forward.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
TAG=divs PAIRS="fp32:base fp32:divs" bash scripts/gpu_micro_ab.sh
