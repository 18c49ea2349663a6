# Interleaved per-step micro-benchmarks: PAIRS="dtype:variant ..." (variant "base" = in-tree build)
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-mab}
mkdir -p $O
for rep in 1 2; do
  for p in $PAIRS; do
    dt=${p%%:*}; v=${p#*:}
    if [ $v = base ]; then so=""; else so="--so build/variants/$v/_C.so"; fi
    timeout -k 10 200 python scripts/micro_step.py --dtype $dt $so --tag ${dt}_$v ${MARGS} >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
  done
done
grep '^{' $O/micro.log | python -c "
import sys, json
for d in map(json.loads, sys.stdin):
    print(d['tag'], {k: v for k, v in d.items() if k not in ('tag', 'dtype')})"
