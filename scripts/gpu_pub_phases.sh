# Rollout phase with / without the published early stop (MACBF_PUBLISH=1/0), headline, 3 rounds.
cd $GRAFT_REPO_ROOT
O=gpurun_out/pubph
mkdir -p $O
for rep in 1 2 3; do
  for v in 1 0; do
    MACBF_PUBLISH=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --phases > $O/b_${v}_$rep.log 2>&1 || { tail -5 $O/b_${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${v}_$rep.log').read().strip().split(chr(10))[-1]); print('publish $v', round(d['ms_per_step'],3), d['phases_ms'])"
  done
done
