#!/bin/bash
# Round 5 batch 6: node16 phase clocks without the dL/dpooled stores (alt_so/nostore, diagnostics);
# kernel trace of the headline with the publication's release removed (alt_so/nofence: the ~6 us
# gap after each controller step); 3-D scan with 8 lanes per agent (alt_so/lpa3): 3-D tests, then
# config #5 fp16 interleaved A/B. Output: gpurun_out/${TAG:-r5b6}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b6}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
MACBF_SELFCHECK=0 MACBF_EXT=alt_so/nostore/_C.so timeout -k 10 200 python scripts/stamps_node.py --node16 --envs 64 > $O/stamps_node16_nostore.log 2>&1 && tail -14 $O/stamps_node16_nostore.log || { echo STOP stamps; exit 1; }
MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/nofence/_C.so TAG=${TAG:-r5b6}/nofence STEPS=6 bash scripts/gpu_prof.sh > $O/nofence_summary.txt 2>&1 || { echo STOP prof; tail -3 $O/nofence_summary.txt; exit 1; }
MACBF_EXT=alt_so/lpa3/_C.so timeout -k 10 300 python -u -m pytest tests/test_gpu_nd.py tests/test_gpu_forward.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/lpa3_tests.log 2>&1
rc=$?; tail -2 $O/lpa3_tests.log; if [ $rc -ne 0 ]; then echo "STOP lpa3 tests"; exit $rc; fi
for rep in 1 2; do
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cfg5_cur_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 cur $rep $(ms $O/cfg5_cur_$rep.log)"
  MACBF_EXT=alt_so/lpa3/_C.so timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cfg5_lpa3_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 lpa3 $rep $(ms $O/cfg5_lpa3_$rep.log)"
done
TAG=r5b7 bash scripts/gpu_r5_b7.sh
