#!/bin/bash
# Interleaved A/B of BASELINE config #2 (32 agents x 1 env) on one box: per-step BPTT launches vs
# the persistent small-scene BPTT (MACBF_SMALL_BPTT), ROUNDS rounds. Output: gpurun_out/${TAG:-ab_cfg2}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_cfg2}
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for v in 0 1; do
    MACBF_SMALL_BPTT=$v timeout -k 10 200 python bench.py --agents 32 --envs 1 --steps 40 --warmup 10 --phases > $O/sb${v}_$r.log 2>&1 || { tail -5 $O/sb${v}_$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/sb${v}_$r.log').read().strip().split(chr(10))[-1]); print('small_bptt=$v', round(d['ms_per_step'],3), d.get('phases_ms'))"
  done
done
