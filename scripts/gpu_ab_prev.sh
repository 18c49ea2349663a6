#!/bin/bash
# A/B of the current build against alt_so/prev/_C.so (the previous build), interleaved on one box;
# optional GPU test subset first (TESTS="tests/test_gpu_node16.py ..."), then node16 phase clocks.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abprev}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; exit $rc; fi
fi
for rep in 1 2 3; do
  for v in new prev; do
    if [ $v = new ]; then E=X=1; else E=MACBF_EXT=alt_so/prev/_C.so; fi
    env $E timeout -k 10 300 python bench.py $ARGS > $O/${v}_${rep}.log 2>&1 || { echo "STOP $v"; exit 1; }
    echo "$v $rep: $(grep '^{' $O/${v}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms")')"
  done
done
timeout -k 10 200 python -u scripts/stamps_node.py --node16 --envs 64 > $O/stamps16.log 2>&1 && tail -14 $O/stamps16.log
