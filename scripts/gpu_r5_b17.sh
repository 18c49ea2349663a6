#!/bin/bash
# Round 5 batch 17: scan culling boxes reduced in registers during the staging (alt_so/boxreg,
# -DSCAN_BOX_REG=1): scan / 3-D / runtime tests (in-tree build too: the staging loop was
# restructured), phase clocks, interleaved headline fp32 x3 and config #5 fp16 x2.
# Output: gpurun_out/${TAG:-r5b17}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b17}
mkdir -p $O
ALT=${ALT:-boxreg}
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_nd.py tests/test_gpu_runtime.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_cur.log 2>&1
rc=$?; tail -1 $O/tests_cur.log; if [ $rc -ne 0 ]; then echo "STOP cur tests"; exit $rc; fi
MACBF_EXT=alt_so/$ALT/_C.so timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_nd.py tests/test_gpu_runtime.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_alt.log 2>&1
rc=$?; tail -1 $O/tests_alt.log; if [ $rc -ne 0 ]; then echo "STOP alt tests"; exit $rc; fi
MACBF_EXT=alt_so/$ALT/_C.so timeout -k 10 200 python scripts/stamps_scan.py > $O/stamps_alt_2d.log 2>&1 && tail -12 $O/stamps_alt_2d.log | head -7 || { echo STOP stamps; exit 1; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/cur_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=alt_so/$ALT/_C.so timeout -k 10 200 python bench.py > $O/alt_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "fp32 $rep cur $(ms $O/cur_fp32_$rep.log) alt $(ms $O/alt_fp32_$rep.log)"
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=alt_so/$ALT/_C.so timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/alt_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 $rep cur $(ms $O/cur_cfg5_$rep.log) alt $(ms $O/alt_cfg5_$rep.log)"
done
