cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_backward.py -q -m gpu -p no:cacheprovider > gpurun_out/r1c_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r1c_tests.log
tail -5 gpurun_out/r1c_tests.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/r1c_bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/r1c_bench.log
tail -3 gpurun_out/r1c_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r1c_prof.log 2>&1
echo "prof rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/r1c_prof.log
tail -3 $GRAFT_REPO_ROOT/gpurun_out/r1c_prof.log
find $GRAFT_REPO_ROOT/gpurun_out/prof1 -name "*stats*" | head
