#!/bin/bash
# A/B of the current build against alt_so/prev/_C.so for the fp32 (x3) and bf16 headlines (REPS
# interleaved pairs each, optional GPU test subset first: TESTS=...), then the 16x16x32 edge
# backward phase clocks of the current build. Output: gpurun_out/${TAG:-abprev2}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abprev2}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; exit $rc; fi
fi
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
for dt in fp32 bf16; do
  for rep in $(seq 1 ${REPS:-2}); do
    for v in new prev; do
      if [ $v = new ]; then E=X=1; else E=MACBF_EXT=alt_so/prev/_C.so; fi
      env $E timeout -k 10 300 python bench.py --dtype $dt $ARGS > $O/${dt}_${v}_${rep}.log 2>&1 || { echo "STOP $dt $v"; tail -3 $O/${dt}_${v}_${rep}.log; exit 1; }
      echo "$dt $v $rep: $(ms $O/${dt}_${v}_${rep}.log) ms"
    done
  done
done
timeout -k 10 300 python scripts/stamps_edge16.py > $O/stamps_edge16.log 2>&1 && grep -v amdgpu.ids $O/stamps_edge16.log
