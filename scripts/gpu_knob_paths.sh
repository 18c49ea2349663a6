# Non-default scheduling paths still run and agree: x3 split controller step, CBF h slices
# overlapped with the rollout, marker + copy early stop (benches: same mean horizon), and the
# runtime tests under the split step. Output: gpurun_out/knobs
cd $GRAFT_REPO_ROOT
O=gpurun_out/knobs
mkdir -p $O
MACBF_X3_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_split.log 2>&1
rc=$?; tail -1 $O/tests_split.log; [ $rc -eq 0 ] || exit $rc
for knobs in "MACBF_X3_SPLIT=1" "MACBF_OVERLAP_HFWD=1" "MACBF_PUBLISH=0" "MACBF_X3_SPLIT=1 MACBF_OVERLAP_HFWD=1"; do
  tag=$(echo $knobs | tr ' =' '__')
  env $knobs timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b_$tag.log 2>&1 || { tail -5 $O/b_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$tag.log').read().strip().split(chr(10))[-1]); print('$knobs', round(d['ms_per_step'],3), 'T', d['mean_T'], 'safety', round(d['safety_rate'],4))"
done
