#!/bin/bash
# Interleaved bench A/B of several builds of the extension on one box: BUILDS="cur alt_so/x/_C.so
# ..." ("cur" = the in-tree build), DTYPES="fp32 bf16", REPS rounds, extra bench flags ARGS,
# optional GPU test subset first (TESTS=..., in-tree build). Output: gpurun_out/${TAG:-abbuilds}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abbuilds}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; exit $rc; fi
fi
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
for dt in ${DTYPES:-fp32 bf16}; do
  for rep in $(seq 1 ${REPS:-2}); do
    n=0
    for b in ${BUILDS:-cur}; do
      n=$((n+1))
      if [ $b = cur ]; then E=X=1; else E=MACBF_EXT=$b; fi
      L=$O/${dt}_b${n}_${rep}.log
      env $E timeout -k 10 300 python bench.py --dtype $dt $ARGS > $L 2>&1 || { echo "STOP $dt $b"; tail -3 $L; exit 1; }
      echo "$dt $b $rep: $(ms $L) ms"
    done
  done
done
