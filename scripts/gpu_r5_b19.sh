#!/bin/bash
# Round 5 batch 19: x3 controller step with double-buffered layer-2 weight fragments (alt_so/wpf,
# -DCTRL_WPF=1; the hoisted bias accumulators dropped for the registers): forward / runtime / fp32
# tests, phase clocks, interleaved headline fp32 x3. Output: gpurun_out/${TAG:-r5b19}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b19}
mkdir -p $O
ALT=${ALT:-wpf}
X=$GRAFT_REPO_ROOT/alt_so/$ALT/_C.so
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
MACBF_EXT=$X timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_runtime.py tests/test_gpu_fp32.py tests/test_gpu_small.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_alt.log 2>&1
rc=$?; tail -1 $O/tests_alt.log; if [ $rc -ne 0 ]; then echo "STOP alt tests"; exit $rc; fi
MACBF_EXT=$X timeout -k 10 200 python scripts/stamps_ctrl.py > $O/stamps_ctrl_alt.log 2>&1 && tail -9 $O/stamps_ctrl_alt.log | head -8 || { echo STOP stamps; exit 1; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/cur_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 200 python bench.py > $O/alt_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "fp32 $rep cur $(ms $O/cur_fp32_$rep.log) alt $(ms $O/alt_fp32_$rep.log)"
done
