# GPU suite (all) -> benches fp32/bf16 -> micro-benchmarks fp32/bf16.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r2b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for d in fp32 bf16; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype $d --phases > $O/bench_$d.log 2>&1 || { tail -5 $O/bench_$d.log; exit 1; }
  tail -1 $O/bench_$d.log | cut -c1-200
  timeout -k 10 300 python scripts/micro_step.py --dtype $d --tag $d > $O/micro_$d.log 2>&1 || { tail -5 $O/micro_$d.log; exit 1; }
  tail -1 $O/micro_$d.log
done
