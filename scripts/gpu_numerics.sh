# Numerics calibration: every rel_cmp comparison of the GPU kernel tests (bf16 vs the emulating
# oracle, fp32 vs the fp32 oracle) logged with its measured error, bounds off, then the summary
cd $GRAFT_REPO_ROOT
O=gpurun_out/numerics
mkdir -p $O
rm -f $O/num.jsonl
MACBF_NUM_LOG=$O/num.jsonl MACBF_NUM_NOASSERT=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_backward.py tests/test_gpu_compat.py tests/test_gpu_nd.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
python scripts/num_summary.py $O/num.jsonl
