#!/bin/bash
# Round 5 batch 16: scan block shapes. 2-D: 512-thread blocks + per-wave count atomics
# (alt_so/d2bswa) vs the default 1024 + barrier; 3-D: 256-thread blocks (alt_so/d3bs256) vs the
# new default 512. Tests per variant, interleaved headline fp32 x3 / config #5 fp16 x2.
# Output: gpurun_out/${TAG:-r5b16}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b16}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
for v in d2bswa d3bs256; do
  MACBF_EXT=alt_so/$v/_C.so timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_nd.py tests/test_gpu_runtime.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; tail -1 $O/tests_$v.log; if [ $rc -ne 0 ]; then echo "STOP $v tests"; exit $rc; fi
done
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/cur_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=alt_so/d2bswa/_C.so timeout -k 10 200 python bench.py > $O/d2bswa_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "fp32 $rep cur $(ms $O/cur_fp32_$rep.log) d2bswa $(ms $O/d2bswa_fp32_$rep.log)"
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=alt_so/d3bs256/_C.so timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/d3bs256_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 $rep cur $(ms $O/cur_cfg5_$rep.log) d3bs256 $(ms $O/d3bs256_cfg5_$rep.log)"
done
