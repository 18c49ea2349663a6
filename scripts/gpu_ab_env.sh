# Interleaved bench A/B over values of one environment knob: VAR=name VALS="a b c"
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abenv}
mkdir -p $O
for rep in 1 2 3; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype ${DT:-fp32} > $O/b_${v}_$rep.log 2>&1 || { tail -5 $O/b_${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${v}_$rep.log').read().strip().split(chr(10))[-1]); print('$VAR=$v $rep', round(d['ms_per_step'],3))"
  done
done
