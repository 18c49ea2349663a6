# fp32 (x3) path: new numerics tests -> full GPU suite -> fp32 + bf16 benches (+ optional rocprof).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-fp32}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/fp32_tests.log 2>&1
rc=$?; tail -3 $O/fp32_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype fp32 --phases > $O/bench_fp32.log 2>&1 || { tail -5 $O/bench_fp32.log; exit 1; }
tail -1 $O/bench_fp32.log | cut -c1-250
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype bf16 --phases > $O/bench_bf16.log 2>&1 || { tail -5 $O/bench_bf16.log; exit 1; }
tail -1 $O/bench_bf16.log | cut -c1-250
if [ "$PROF" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --dtype fp32 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
  echo "prof rc=$?"
fi
