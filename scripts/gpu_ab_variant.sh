# A/B of a kernel change: GPU backward/runtime tests on the in-tree build, then interleaved
# per-step micro-benchmarks (variant $OLD vs in-tree), then the headline bench. Output: gpurun_out/$TAG
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/${TAG:-tail}
O=gpurun_out/${TAG:-tail}
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_runtime.py tests/test_gpu_dp.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python scripts/micro_step.py --so build/variants/${OLD:-oldtail}/_C.so --tag old$rep >> $O/micro.log 2>&1 || exit 1
  timeout -k 10 300 python scripts/micro_step.py --tag new$rep >> $O/micro.log 2>&1 || exit 1
done
grep -v "^\s*$" $O/micro.log | tail -8
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
