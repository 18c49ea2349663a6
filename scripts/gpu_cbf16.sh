#!/bin/bash
# 16x16x32 x3 CBF backward: the GPU test suite (TESTS overrides), the new-vs-old kernel check, the
# active-list micro-benchmark of the new kernel and of the 32x32x16 kernel (MACBF_CBF16=0), phase
# clocks, then the headline bench. Output: gpurun_out/${TAG:-cbf16}
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cbf16}
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/check_cbf16.py > $O/chk.log 2>&1 && tail -1 $O/chk.log | cut -c1-300 || exit 1
timeout -k 10 200 python scripts/micro_cbfbwd.py --tag cbf16 > $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
tail -1 $O/micro.log
MACBF_CBF16=0 timeout -k 10 200 python scripts/micro_cbfbwd.py --tag cbf32 >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
tail -1 $O/micro.log
timeout -k 10 200 python scripts/stamps_cbf.py > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 1; }
tail -1 $O/stamps.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
MACBF_CBF16=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_cbf32.log 2>&1 || { tail -5 $O/bench_cbf32.log; exit 1; }
tail -1 $O/bench_cbf32.log | cut -c1-300
