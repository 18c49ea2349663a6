cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -E "gfx950|Compute Unit" | head -4 > gpurun_out/g1_info.txt
timeout -k 10 900 python -m pytest tests/test_gpu_probe.py tests/test_gpu_forward.py -q -m gpu -p no:cacheprovider > gpurun_out/g1_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/g1_tests.log
tail -30 gpurun_out/g1_tests.log
