#!/bin/bash
# 16x16x32 x3 CBF backward: layout probe + CBF / full-step numerics tests, then the active-list
# micro-benchmark of the new kernel and of the 32x32x16 kernel (MACBF_CBF16=0) and the new
# kernel's phase clocks. Output: gpurun_out/${TAG:-cbf16}
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cbf16}
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_probe.py tests/test_gpu_dedup.py tests/test_gpu_fp32.py} -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
MACBF_CBF16=1 timeout -k 10 200 python scripts/micro_cbfbwd.py --tag cbf16 > $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
tail -1 $O/micro.log
MACBF_CBF16=0 timeout -k 10 200 python scripts/micro_cbfbwd.py --tag cbf32 >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
tail -1 $O/micro.log
MACBF_CBF16=1 timeout -k 10 200 python scripts/stamps_cbf.py > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 1; }
tail -1 $O/stamps.log
