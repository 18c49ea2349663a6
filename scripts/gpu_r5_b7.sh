#!/bin/bash
# Round 5 batch 7: node16 dL/dpooled stores from tile pairs (alt_so/dppair): node / full-step tests
# with the variant, its phase clocks, interleaved headline A/B (fp32, bf16). Output: gpurun_out/${TAG:-r5b7}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b7}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
MACBF_EXT=alt_so/dppair/_C.so timeout -k 10 400 python -u -m pytest tests/test_gpu_node16.py tests/test_gpu_fp32.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/dppair_tests.log 2>&1
rc=$?; tail -2 $O/dppair_tests.log; if [ $rc -ne 0 ]; then echo "STOP dppair tests"; exit $rc; fi
MACBF_EXT=alt_so/dppair/_C.so timeout -k 10 200 python scripts/stamps_node.py --node16 --envs 64 > $O/stamps_dppair.log 2>&1 && tail -6 $O/stamps_dppair.log
for rep in 1 2 3; do
  for dt in fp32 bf16; do
    timeout -k 10 200 python bench.py --dtype $dt > $O/cur_${dt}_$rep.log 2>&1 || { echo STOP; exit 1; }
    MACBF_EXT=alt_so/dppair/_C.so timeout -k 10 200 python bench.py --dtype $dt > $O/dppair_${dt}_$rep.log 2>&1 || { echo STOP; exit 1; }
    echo "$dt $rep cur $(ms $O/cur_${dt}_$rep.log) dppair $(ms $O/dppair_${dt}_$rep.log)"
  done
done
