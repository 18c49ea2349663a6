#!/bin/bash
# Round 5 batch 1: per-env horizons of the headline (scripts/diag_horizons.py); the early-stop
# publication without its system-scope release (alt_so/nofence) -- runtime tests + interleaved
# bench A/B; the fused node+edge BPTT step at the headline (32-agent chunks, VERDICT r4 item 1
# fallback) vs the default 16x16x32 node / edge launches. Output: gpurun_out/${TAG:-r5b1}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b1}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
timeout -k 10 200 python scripts/diag_horizons.py --iters 25 > $O/horizons.jsonl 2> $O/horizons.err || { echo "STOP horizons"; tail -3 $O/horizons.err; exit 1; }
tail -1 $O/horizons.jsonl
MACBF_EXT=alt_so/nofence/_C.so timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/nofence_tests.log 2>&1
rc=$?; tail -2 $O/nofence_tests.log; if [ $rc -ne 0 ]; then echo "STOP nofence tests"; exit $rc; fi
for rep in 1 2; do
  timeout -k 10 200 python bench.py > $O/cur_$rep.log 2>&1 || { echo STOP; tail -3 $O/cur_$rep.log; exit 1; }
  echo "cur $rep $(ms $O/cur_$rep.log)"
  MACBF_EXT=alt_so/nofence/_C.so timeout -k 10 200 python bench.py > $O/nofence_$rep.log 2>&1 || { echo STOP; tail -3 $O/nofence_$rep.log; exit 1; }
  echo "nofence $rep $(ms $O/nofence_$rep.log)"
  MACBF_NODE_CHUNK=32 MACBF_BWD_FUSED=1 timeout -k 10 200 python bench.py > $O/fused32_$rep.log 2>&1 || { echo STOP; tail -3 $O/fused32_$rep.log; exit 1; }
  echo "fused32 $rep $(ms $O/fused32_$rep.log)"
done
