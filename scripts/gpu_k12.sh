# Edge backward with compile-time K = 12 vs runtime K (MACBF_EB_K12=0): backward GPU tests, then
# interleaved per-step micro-benchmark + headline bench. Output: gpurun_out/k12
cd $GRAFT_REPO_ROOT
O=gpurun_out/k12
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32.py tests/test_gpu_backward.py tests/test_gpu_nd.py tests/test_gpu_runtime.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    MACBF_EB_K12=$v timeout -k 10 300 python scripts/micro_step.py --tag k12_${v}_$rep >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
    MACBF_EB_K12=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_${v}_$rep.log 2>&1 || { tail -5 $O/b_${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${v}_$rep.log').read().strip().split(chr(10))[-1]); print('k12 $v', round(d['ms_per_step'],3))"
  done
done
grep '^{' $O/micro.log | cut -c1-220
