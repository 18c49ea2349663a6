#!/bin/bash
# Round 5: GPU suite on the in-tree build, then an interleaved headline A/B of the in-tree build
# against alt_so/$ALT (REPS rounds, bench ARGS). Output: gpurun_out/${TAG:-r5ab}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5ab}
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -4 $O/gpu_tests.log
  if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; exit $rc; fi
fi
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
for rep in $(seq 1 ${REPS:-2}); do
  timeout -k 10 200 python bench.py $ARGS > $O/new_$rep.log 2>&1 || { echo STOP; tail -3 $O/new_$rep.log; exit 1; }
  echo "new $rep $(ms $O/new_$rep.log)"
  MACBF_EXT=alt_so/$ALT/_C.so timeout -k 10 200 python bench.py $ARGS > $O/old_$rep.log 2>&1 || { echo STOP; tail -3 $O/old_$rep.log; exit 1; }
  echo "old $rep $(ms $O/old_$rep.log)"
done
