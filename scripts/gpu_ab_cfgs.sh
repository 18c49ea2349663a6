# Interleaved bench A/B over named env configurations: CFGS="name1:VAR=a,VAR2=b name2:..."
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abcfg}
mkdir -p $O
for rep in 1 2 3; do
  for c in $CFGS; do
    name=${c%%:*}; vars=${c#*:}
    env $(echo $vars | tr ',' ' ') timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype ${DT:-fp32} --phases > $O/b_${name}_$rep.log 2>&1 || { tail -5 $O/b_${name}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${name}_$rep.log').read().strip().split(chr(10))[-1]); p=d.get('phases_ms',{}); print('$name $rep', round(d['ms_per_step'],3), 'rollout', p.get('rollout'), 'cbf', p.get('cbf'))"
  done
done
