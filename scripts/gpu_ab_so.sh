#!/bin/bash
# Interleaved per-kernel micro-benchmarks (scripts/micro_step.py) of the in-tree extension vs an
# alternative build: ALT=path/to/_C.so ARGS="micro_step args" ROUNDS=2 -> gpurun_out/${TAG:-ab_so}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_so}
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  timeout -k 10 200 python scripts/micro_step.py --tag new $ARGS > $O/new_$r.log 2>&1 || { tail -5 $O/new_$r.log; exit 1; }
  tail -1 $O/new_$r.log
  timeout -k 10 200 python scripts/micro_step.py --tag alt --so $ALT $ARGS > $O/alt_$r.log 2>&1 || { tail -5 $O/alt_$r.log; exit 1; }
  tail -1 $O/alt_$r.log
done
