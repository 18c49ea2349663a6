#!/bin/bash
# Round 5 batch 4: fixed-horizon headline (T = 50, no early stop: no per-step publication, no host
# poll) -- bench fp32 / bf16 and a kernel trace, to separate the per-step gap after the controller
# step from the early-stop mechanism. Output: gpurun_out/${TAG:-r5b4}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b4}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
for dt in fp32 bf16; do
  timeout -k 10 300 python bench.py --no_early_stop --dtype $dt > $O/fixedT_$dt.log 2>&1 || { echo STOP; tail -3 $O/fixedT_$dt.log; exit 1; }
  echo "fixedT $dt $(ms $O/fixedT_$dt.log)"
done
TAG=${TAG:-r5b4}/fixedT STEPS=4 ARGS="--no_early_stop" bash scripts/gpu_prof.sh > $O/fixedT_summary.txt 2>&1 && head -8 $O/fixedT_summary.txt
