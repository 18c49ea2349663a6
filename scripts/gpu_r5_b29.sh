#!/bin/bash
# Round 5 batch 29: cell-grid scatter from the counting pass's atomic ranks (one LDS atomic pass
# instead of two) + cell-path counters in the phase clocks. in-tree vs alt_so/prev (HEAD). Tests,
# 2-D / 3-D phase clocks, interleaved headline fp32 x2 and config #5 fp16 x2.
# Output: gpurun_out/${TAG:-r5b29}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b29}
mkdir -p $O
P=$GRAFT_REPO_ROOT/alt_so/prev/_C.so
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
T="tests/test_gpu_nd.py tests/test_gpu_forward.py tests/test_gpu_runtime.py tests/test_gpu_small.py"
timeout -k 10 400 python -u -m pytest $T -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_cur.log 2>&1
rc=$?; tail -1 $O/tests_cur.log; if [ $rc -ne 0 ]; then echo "STOP cur tests"; exit $rc; fi
timeout -k 10 200 python scripts/stamps_scan.py > $O/stamps_cur_2d.log 2>&1 && tail -14 $O/stamps_cur_2d.log | head -13 || { echo STOP stamps; exit 1; }
timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_cur_3d.log 2>&1 && tail -14 $O/stamps_cur_3d.log | head -13 || { echo STOP stamps; exit 1; }
for rep in 1 2; do
  MACBF_EXT=$P timeout -k 10 200 python bench.py > $O/prev_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  timeout -k 10 200 python bench.py > $O/cur_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "fp32 $rep prev $(ms $O/prev_fp32_$rep.log) cur $(ms $O/cur_fp32_$rep.log)"
done
for rep in 1 2; do
  MACBF_EXT=$P timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/prev_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 fp16 $rep prev $(ms $O/prev_cfg5_$rep.log) cur $(ms $O/cur_cfg5_$rep.log)"
done
