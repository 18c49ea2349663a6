# Scan lane layouts: GPU tests (forward / large / runtime), then interleaved headline A/B of the
# per-step micro-benchmark: default (4 lanes, 1024-thread blocks), 8 lanes in 256-thread blocks
# (MACBF_SCAN_LPA8=1) and 8 lanes in 1024-thread blocks (build/variants/lpa8big). Output: gpurun_out/lanes
cd $GRAFT_REPO_ROOT
O=gpurun_out/lanes
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_large.py tests/test_gpu_runtime.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python scripts/micro_step.py --tag base_$rep >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
  MACBF_SCAN_LPA8=1 timeout -k 10 300 python scripts/micro_step.py --tag lpa8small_$rep >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
  MACBF_EXT=$GRAFT_REPO_ROOT/build/variants/lpa8big/_C.so timeout -k 10 300 python scripts/micro_step.py --so build/variants/lpa8big/_C.so --tag lpa8big_$rep >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
done
grep '^{' $O/micro.log | cut -c1-200
