#!/bin/bash
# Round 5 batch 35: cell prefix sum over PC cells per thread (grids with more cells than block
# threads). alt_so/pc8 = that with the 8^3 3-D grid (same grid as in-tree), alt_so/g10 / g12 =
# 10^3 / 12^3 cells in the 512-thread 3-D blocks. Tests, 3-D phase clocks, interleaved config #5
# fp16 x2 and headline fp32 x1. Output: gpurun_out/${TAG:-r5b35}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b35}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
T="tests/test_gpu_nd.py tests/test_gpu_forward.py tests/test_gpu_runtime.py tests/test_gpu_small.py"
for v in pc8 g10 g12; do
  MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$v/_C.so timeout -k 10 400 python -u -m pytest $T -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v $(tail -n 1 $O/tests_$v.log)"; if [ $rc -ne 0 ]; then echo "STOP $v tests"; exit $rc; fi
done
for v in g10 g12; do
  MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$v/_C.so timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_${v}_3d.log 2>&1 && tail -n 14 $O/stamps_${v}_3d.log | head -13 || { echo STOP stamps; exit 1; }
done
for rep in 1 2; do
  line="cfg5 fp16 $rep"
  for v in cur pc8 g10 g12; do
    if [ $v = cur ]; then E=; else E=$GRAFT_REPO_ROOT/alt_so/$v/_C.so; fi
    MACBF_EXT=$E timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/${v}_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
    line="$line $v $(ms $O/${v}_cfg5_$rep.log)"
  done
  echo "$line"
done
timeout -k 10 200 python bench.py > $O/cur_fp32.log 2>&1 || { echo STOP; exit 1; }
MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/pc8/_C.so timeout -k 10 200 python bench.py > $O/pc8_fp32.log 2>&1 || { echo STOP; exit 1; }
echo "fp32 cur $(ms $O/cur_fp32.log) pc8 $(ms $O/pc8_fp32.log)"
