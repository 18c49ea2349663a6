# EB_WLS1 check: x3 edge-backward tests, then interleaved micro A/B against the shared-S1 build
cd $GRAFT_REPO_ROOT
O=gpurun_out/wls1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp32.py tests/test_gpu_backward.py tests/test_gpu_small.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
TAG=wls1 PAIRS="fp32:base fp32:nowls1" bash scripts/gpu_micro_ab.sh
