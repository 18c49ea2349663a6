#!/bin/bash
# Round 5 batch 28: 3-D cell grid shape A/B at config #5 (fp16): in-tree (8^3 cells, 512-thread
# blocks) vs alt_so/g6 (6^3), alt_so/g7 (7^3), alt_so/b1k (8^3, 1024-thread blocks); nd tests of each,
# interleaved x2, 3-D phase clocks of the in-tree build. Output: gpurun_out/${TAG:-r5b28}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b28}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_nd.py tests/test_gpu_forward.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_cur.log 2>&1
rc=$?; tail -1 $O/tests_cur.log; if [ $rc -ne 0 ]; then echo "STOP cur tests"; exit $rc; fi
for v in g6 g7 b1k; do
  MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$v/_C.so timeout -k 10 300 python -u -m pytest tests/test_gpu_nd.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v $(tail -1 $O/tests_$v.log)"; if [ $rc -ne 0 ]; then echo "STOP $v tests"; exit $rc; fi
done
timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_cur_3d.log 2>&1 && tail -14 $O/stamps_cur_3d.log || { echo STOP stamps; exit 1; }
for rep in 1 2; do
  line="cfg5 fp16 $rep"
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  line="$line cur $(ms $O/cur_cfg5_$rep.log)"
  for v in g6 g7 b1k; do
    MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$v/_C.so timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/${v}_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
    line="$line $v $(ms $O/${v}_cfg5_$rep.log)"
  done
  echo "$line"
done
