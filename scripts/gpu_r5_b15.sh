#!/bin/bash
# Round 5 batch 15: 3-D scan block imbalance: 512-thread blocks (two per CU) for 3-D scenes
# (alt_so/d3bs) and additionally per-wave count atomics (alt_so/d3bswa). 3-D tests per variant,
# interleaved config #5 fp16 x2 and fp32 x1, 3-D phase clocks of d3bswa.
# Output: gpurun_out/${TAG:-r5b15}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b15}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
for v in d3bs d3bswa; do
  MACBF_EXT=alt_so/$v/_C.so timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_nd.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; tail -1 $O/tests_$v.log; if [ $rc -ne 0 ]; then echo "STOP $v tests"; exit $rc; fi
done
for rep in 1 2; do
  for v in cur d3bs d3bswa; do
    if [ $v != cur ]; then E="MACBF_EXT=alt_so/$v/_C.so"; else E=""; fi
    env $E timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/${v}_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  done
  echo "cfg5 fp16 $rep cur $(ms $O/cur_cfg5_$rep.log) d3bs $(ms $O/d3bs_cfg5_$rep.log) d3bswa $(ms $O/d3bswa_cfg5_$rep.log)"
done
for v in cur d3bs d3bswa; do
  if [ $v != cur ]; then E="MACBF_EXT=alt_so/$v/_C.so"; else E=""; fi
  env $E timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 > $O/${v}_cfg5_fp32.log 2>&1 || { echo STOP; exit 1; }
done
echo "cfg5 fp32 cur $(ms $O/cur_cfg5_fp32.log) d3bs $(ms $O/d3bs_cfg5_fp32.log) d3bswa $(ms $O/d3bswa_cfg5_fp32.log)"
MACBF_EXT=alt_so/d3bswa/_C.so timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_scan_3d_d3bswa.log 2>&1 && tail -12 $O/stamps_scan_3d_d3bswa.log
