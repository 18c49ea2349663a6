# Strong-scaling slice (1024 agents x ENVS envs per GPU) benches over env configurations CFGS
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-slice}
mkdir -p $O
for rep in 1 2; do
  for c in $CFGS; do
    name=${c%%:*}; vars=${c#*:}
    env $(echo $vars | tr ',' ' ') timeout -k 10 300 python bench.py --envs ${ENVS:-8} --steps 20 --warmup 3 --dtype ${DT:-fp32} --phases > $O/b_${name}_$rep.log 2>&1 || { tail -5 $O/b_${name}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${name}_$rep.log').read().strip().split(chr(10))[-1]); p=d.get('phases_ms',{}); print('$name $rep', round(d['ms_per_step'],3), 'rollout', p.get('rollout'), 'cbf', p.get('cbf'), 'bptt', p.get('bptt'))"
  done
done
