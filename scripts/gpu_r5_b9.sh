#!/bin/bash
# Round 5 batch 9: CBF backward weight-gradient stages in four 32-row turns
# through two alternating buffers, one barrier per turn (alt_so/cbfdb, -DCBF16_DB=1): oracle and
# full-step tests with the variant, its phase clocks, interleaved headline A/B (fp32 x3, bf16 x2).
# Output: gpurun_out/${TAG:-r5b9}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b9}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
MACBF_EXT=alt_so/cbfdb/_C.so timeout -k 10 400 python -u -m pytest tests/test_gpu_oracle16.py tests/test_gpu_fp32.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/cbfdb_tests.log 2>&1
rc=$?; tail -2 $O/cbfdb_tests.log; if [ $rc -ne 0 ]; then echo "STOP cbfdb tests"; exit $rc; fi
timeout -k 10 200 python scripts/stamps_cbf.py --envs 64 > $O/stamps_cbf_cur.log 2>&1 && tail -8 $O/stamps_cbf_cur.log || { echo STOP stamps; exit 1; }
MACBF_EXT=alt_so/cbfdb/_C.so timeout -k 10 200 python scripts/stamps_cbf.py --envs 64 > $O/stamps_cbf_db.log 2>&1 && tail -8 $O/stamps_cbf_db.log || { echo STOP stamps; exit 1; }
for rep in 1 2 3; do
  for dt in fp32 bf16; do
    if [ $dt = bf16 ] && [ $rep = 3 ]; then continue; fi
    timeout -k 10 200 python bench.py --dtype $dt > $O/cur_${dt}_$rep.log 2>&1 || { echo STOP; exit 1; }
    MACBF_EXT=alt_so/cbfdb/_C.so timeout -k 10 200 python bench.py --dtype $dt > $O/db_${dt}_$rep.log 2>&1 || { echo STOP; exit 1; }
    echo "$dt $rep cur $(ms $O/cur_${dt}_$rep.log) db $(ms $O/db_${dt}_$rep.log)"
  done
done
