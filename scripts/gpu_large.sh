# Large envs (> 4096 nodes): GPU tests -> bench 16384 agents x 4 envs (fp32, bf16) -> full GPU suite.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-large}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/large_tests.log 2>&1
rc=$?; tail -3 $O/large_tests.log; [ $rc -eq 0 ] || exit $rc
for d in fp32 bf16; do
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 --dtype $d --agents 16384 --envs 4 --phases > $O/bench16k_$d.log 2>&1 || { tail -5 $O/bench16k_$d.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench16k_$d.log').read().strip().split(chr(10))[-1]); print('$d', round(d['ms_per_step'],2), round(d['value']/1e6,2), d['mean_T'], d.get('phases_ms'))"
done
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; exit $rc
