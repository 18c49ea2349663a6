#!/bin/bash
# Interleaved A/B of an environment setting on one box: bench.py $ARGS with $ENV_A vs $ENV_B, $REPS
# repetitions; optional GPU test subset first (TESTS=...). Output: gpurun_out/${TAG:-abenv}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abenv}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; exit $rc; fi
fi
for rep in $(seq 1 ${REPS:-3}); do
  for v in A B; do
    if [ $v = A ]; then E=${ENV_A:-X=1}; else E=${ENV_B:-X=1}; fi
    env $E timeout -k 10 300 python bench.py $ARGS > $O/${v}_${rep}.log 2>&1 || { echo "STOP $v"; tail -3 $O/${v}_${rep}.log; exit 1; }
    echo "$v ($E) $rep: $(grep '^{' $O/${v}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms T", d["mean_T"])')"
  done
done
