#!/bin/bash
# Round 5 batch 31: cell-row table (the agent's lanes compute the ranges of 16 rows at once into
# LDS before the candidate loop) = alt_so/rowtab, vs in-tree (rows advanced inside the loop);
# alt_so/rtv3 = rowtab + cell records carrying the node's speed (SCAN_CELL_VZ=1: no dependent
# velocity read for the safety pre-test). Tests, phase clocks, interleaved headline fp32 x2 and
# config #5 fp16 x2. Output: gpurun_out/${TAG:-r5b31}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b31}
mkdir -p $O
X=$GRAFT_REPO_ROOT/alt_so/rowtab/_C.so
V=$GRAFT_REPO_ROOT/alt_so/rtv3/_C.so
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
T="tests/test_gpu_nd.py tests/test_gpu_forward.py tests/test_gpu_runtime.py tests/test_gpu_small.py"
MACBF_EXT=$X timeout -k 10 400 python -u -m pytest $T -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_rowtab.log 2>&1
rc=$?; tail -1 $O/tests_rowtab.log; if [ $rc -ne 0 ]; then echo "STOP rowtab tests"; exit $rc; fi
MACBF_EXT=$V timeout -k 10 400 python -u -m pytest $T -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_rtv3.log 2>&1
rc=$?; tail -1 $O/tests_rtv3.log; if [ $rc -ne 0 ]; then echo "STOP rtv3 tests"; exit $rc; fi
MACBF_EXT=$X timeout -k 10 200 python scripts/stamps_scan.py > $O/stamps_rowtab_2d.log 2>&1 && tail -14 $O/stamps_rowtab_2d.log | head -7 || { echo STOP stamps; exit 1; }
MACBF_EXT=$V timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_rtv3_3d.log 2>&1 && tail -14 $O/stamps_rtv3_3d.log | head -13 || { echo STOP stamps; exit 1; }
for rep in 1 2; do
  timeout -k 10 200 python bench.py > $O/cur_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 200 python bench.py > $O/rowtab_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$V timeout -k 10 200 python bench.py > $O/rtv3_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "fp32 $rep cur $(ms $O/cur_fp32_$rep.log) rowtab $(ms $O/rowtab_fp32_$rep.log) rtv3 $(ms $O/rtv3_fp32_$rep.log)"
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/rowtab_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$V timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/rtv3_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 fp16 $rep cur $(ms $O/cur_cfg5_$rep.log) rowtab $(ms $O/rowtab_cfg5_$rep.log) rtv3 $(ms $O/rtv3_cfg5_$rep.log)"
done
