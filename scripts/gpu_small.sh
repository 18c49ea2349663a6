# Persistent small-scene rollout: GPU tests, then config #2 benches (32 agents x 1 env) with the
# persistent rollout on / off, and a kernel trace of the 32 x 1 iteration. Output: gpurun_out/${TAG:-small}
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-small}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py ${EXTRA_TESTS} -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for dt in fp32 bf16; do
  for sm in 1 0; do
    MACBF_SMALL_ROLLOUT=$sm timeout -k 10 300 python bench.py --agents 32 --envs 1 --steps 30 --warmup 5 --dtype $dt --phases > $O/cfg2_${dt}_small$sm.log 2>&1 || { tail -5 $O/cfg2_${dt}_small$sm.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/cfg2_${dt}_small$sm.log').read().strip().split(chr(10))[-1]); print('$dt small=$sm', round(d['ms_per_step'],3), round(d['value']/1e6,3), d.get('phases_ms'))"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --agents 32 --envs 1 --steps 5 --warmup 2 --dtype fp32 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
