cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_probe.py tests/test_gpu_forward.py tests/test_gpu_backward.py -q -m gpu -p no:cacheprovider > gpurun_out/r1d_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r1d_tests.log
tail -6 gpurun_out/r1d_tests.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/r1d_bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/r1d_bench.log
tail -2 gpurun_out/r1d_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r1d_prof.log 2>&1
echo "prof rc=$?"
