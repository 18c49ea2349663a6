#!/bin/bash
# Round 5 batch 11: controller step with the dense pool interleaved into the edge MLP's MFMA chains
# (alt_so/poolil, -DCTRL_POOL_IL=1): forward / runtime / fp32 tests with the variant, phase clocks of
# both builds, interleaved headline A/B (fp32 x3, bf16 x2). Output: gpurun_out/${TAG:-r5b11}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b11}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
MACBF_EXT=alt_so/${ALT:-poolil}/_C.so timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_runtime.py tests/test_gpu_fp32.py tests/test_gpu_small.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/alt_tests.log 2>&1
rc=$?; tail -2 $O/alt_tests.log; if [ $rc -ne 0 ]; then echo "STOP alt tests"; exit $rc; fi
timeout -k 10 200 python scripts/stamps_ctrl.py > $O/stamps_cur.log 2>&1 && tail -9 $O/stamps_cur.log | head -8 || { echo STOP stamps; exit 1; }
MACBF_EXT=alt_so/${ALT:-poolil}/_C.so timeout -k 10 200 python scripts/stamps_ctrl.py > $O/stamps_alt.log 2>&1 && tail -9 $O/stamps_alt.log | head -8 || { echo STOP stamps; exit 1; }
for rep in 1 2 3; do
  for dt in fp32 bf16; do
    if [ $dt = bf16 ] && [ $rep = 3 ]; then continue; fi
    timeout -k 10 200 python bench.py --dtype $dt > $O/cur_${dt}_$rep.log 2>&1 || { echo STOP; exit 1; }
    MACBF_EXT=alt_so/${ALT:-poolil}/_C.so timeout -k 10 200 python bench.py --dtype $dt > $O/alt_${dt}_$rep.log 2>&1 || { echo STOP; exit 1; }
    echo "$dt $rep cur $(ms $O/cur_${dt}_$rep.log) alt $(ms $O/alt_${dt}_$rep.log)"
  done
done
