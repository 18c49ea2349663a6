# Scan with 8 lanes per agent for small grids: forward/large/small GPU tests, then interleaved
# A/B (MACBF_SCAN_LPA8=0/1) of the 8-env and 16-env strong-scaling slices. Output: gpurun_out/lpa8
cd $GRAFT_REPO_ROOT
O=gpurun_out/lpa8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_large.py tests/test_gpu_nd.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 0 1; do
    for e in 8 16; do
      MACBF_SCAN_LPA8=$v timeout -k 10 200 python bench.py --envs $e --steps 10 --warmup 3 --phases > $O/b_${e}_${v}_${rep}.log 2>&1 || { tail -5 $O/b_${e}_${v}_${rep}.log; exit 1; }
      python -c "import json; d=json.loads(open('$O/b_${e}_${v}_${rep}.log').read().strip().split(chr(10))[-1]); print('envs $e lpa8=$v', round(d['ms_per_step'],3), d.get('phases_ms',{}).get('rollout'))"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
MACBF_SCAN_LPA8=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --envs 8 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof8.log 2>&1 || exit 1
