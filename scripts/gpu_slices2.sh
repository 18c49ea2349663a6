# Strong-scaling per-rank slices of the 64-env config (32 / 16 / 8 envs per GPU) + GPU tests
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-slices}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for dt in fp32 bf16; do
  for e in 32 16 8; do
    timeout -k 10 300 python bench.py --envs $e --steps 20 --warmup 3 --dtype $dt --phases > $O/slice_${dt}_$e.log 2>&1 || { tail -5 $O/slice_${dt}_$e.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/slice_${dt}_$e.log').read().strip().split(chr(10))[-1]); print('$dt $e envs', round(d['ms_per_step'],3), round(d['value']/1e6,2), d['config'].get('global_batch'), d.get('scaling'))"
  done
done
