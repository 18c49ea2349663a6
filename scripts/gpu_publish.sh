# Published early stop (ctrl.hip publish_step): runtime / small / backward GPU tests, smoke, then
# interleaved A/B (MACBF_PUBLISH=0/1) of the headline bench and the 8-env slice. Output: gpurun_out/pub
cd $GRAFT_REPO_ROOT
O=gpurun_out/pub
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_small.py tests/test_gpu_fp32.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
for rep in 1 2; do
  for v in 0 1; do
    MACBF_PUBLISH=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_${v}_$rep.log 2>&1 || { tail -5 $O/b_${v}_$rep.log; exit 1; }
    MACBF_PUBLISH=$v timeout -k 10 300 python bench.py --envs 8 --steps 10 --warmup 3 --phases > $O/s8_${v}_$rep.log 2>&1 || { tail -5 $O/s8_${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${v}_$rep.log').read().strip().split(chr(10))[-1]); e=json.loads(open('$O/s8_${v}_$rep.log').read().strip().split(chr(10))[-1]); print('publish $v headline', round(d['ms_per_step'],3), 'T', d['mean_T'], 'slice8', round(e['ms_per_step'],3), e['phases_ms']['rollout'])"
  done
done
