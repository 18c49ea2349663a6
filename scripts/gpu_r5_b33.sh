#!/bin/bash
# Round 5 batch 33: 2-D cell grid resolution with the row-table walk: in-tree 16^2 vs alt_so/g24
# (24^2) and alt_so/g32 (32^2). Tests of each, phase clocks, interleaved headline fp32 x2.
# Output: gpurun_out/${TAG:-r5b33}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b33}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
for v in g24 g32; do
  MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$v/_C.so timeout -k 10 300 python -u -m pytest tests/test_gpu_nd.py tests/test_gpu_forward.py tests/test_gpu_runtime.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v $(tail -n 1 $O/tests_$v.log)"; if [ $rc -ne 0 ]; then echo "STOP $v tests"; exit $rc; fi
  MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$v/_C.so timeout -k 10 200 python scripts/stamps_scan.py > $O/stamps_${v}_2d.log 2>&1 && tail -n 14 $O/stamps_${v}_2d.log | head -13 || { echo STOP stamps; exit 1; }
done
for rep in 1 2; do
  line="fp32 $rep"
  for v in cur g24 g32; do
    if [ $v = cur ]; then E=; else E=$GRAFT_REPO_ROOT/alt_so/$v/_C.so; fi
    MACBF_EXT=$E timeout -k 10 200 python bench.py > $O/${v}_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
    line="$line $v $(ms $O/${v}_fp32_$rep.log)"
  done
  echo "$line"
done
