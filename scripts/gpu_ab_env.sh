#!/bin/bash
# Interleaved A/B of an environment knob on one box: VAR=NAME VALS="0 1" ARGS="bench args"
# ROUNDS=2 -> gpurun_out/${TAG:-ab_env}/NAME_<val>_<round>.log and one summary line per run.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_env}
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VALS:-0 1}; do
    f=$O/${VAR}_${v}_$r.log
    env $VAR=$v timeout -k 10 200 python bench.py $ARGS --phases > $f 2>&1 || { tail -5 $f; exit 1; }
    python -c "import json; d=json.loads(open('$f').read().strip().split(chr(10))[-1]); print('$VAR=$v', round(d['ms_per_step'],3), d.get('phases_ms'))"
  done
done
