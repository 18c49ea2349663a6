# GPU validation of the backward kernels + first bench + profile. Each GPU step has its own limit.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_probe.py tests/test_gpu_forward.py tests/test_gpu_backward.py -q -m gpu -p no:cacheprovider > gpurun_out/r1b_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r1b_tests.log
tail -40 gpurun_out/r1b_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/r1b_bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/r1b_bench.log
tail -5 gpurun_out/r1b_bench.log
