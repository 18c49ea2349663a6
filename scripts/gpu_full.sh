# Full GPU test suite (one process) + headline bench + kernel trace. Output: gpurun_out/${TAG:-full}
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-full}
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --phases > $O/bench_fp32.log 2>&1 || { tail -5 $O/bench_fp32.log; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype bf16 --phases > $O/bench_bf16.log 2>&1 || { tail -5 $O/bench_bf16.log; exit 1; }
for f in bench_fp32 bench_bf16; do python -c "import json; d=json.loads(open('$O/$f.log').read().strip().split(chr(10))[-1]); print('$f', round(d['ms_per_step'],3), round(d['value']/1e6,2), d.get('phases_ms'))"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
