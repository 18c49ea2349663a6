# Correctness + perf check after a kernel change: the named GPU test files, per-step micro
# benchmarks (headline and 32 x 1), headline bench and config #2 bench (fp32 unless DT is set).
# Output: gpurun_out/${TAG:-chk}
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-chk}
mkdir -p $O
DT=${DT:-fp32}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_small.py tests/test_gpu_fp32.py tests/test_gpu_backward.py} -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/micro_step.py --dtype $DT --tag $TAG > $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
timeout -k 10 300 python scripts/micro_step.py --dtype $DT --agents 32 --envs 1 --tag ${TAG}_32x1 >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
grep '^{' $O/micro.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype $DT --phases > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
timeout -k 10 300 python bench.py --agents 32 --envs 1 --steps 30 --warmup 5 --dtype $DT --phases > $O/cfg2.log 2>&1 || { tail -5 $O/cfg2.log; exit 1; }
for f in bench cfg2; do python -c "import json; d=json.loads(open('$O/$f.log').read().strip().split(chr(10))[-1]); print('$f', round(d['ms_per_step'],3), round(d['value']/1e6,3), d.get('phases_ms'))"; done
