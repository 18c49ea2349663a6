# Edge-backward grid A/B: workgroups per CU cap 2 (default; x3 holds one per CU) vs 1
# (MACBF_EDGE_WG_PER_CU): per-step micro-benchmark + headline bench, interleaved. Output: gpurun_out/egrid
cd $GRAFT_REPO_ROOT
O=gpurun_out/egrid
mkdir -p $O
for rep in 1 2; do
  for v in 2 1; do
    MACBF_EDGE_WG_PER_CU=$v timeout -k 10 300 python scripts/micro_step.py --tag wgpc${v}_$rep >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
    MACBF_EDGE_WG_PER_CU=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b_${v}_$rep.log 2>&1 || { tail -5 $O/b_${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${v}_$rep.log').read().strip().split(chr(10))[-1]); print('wg/cu $v', round(d['ms_per_step'],3))"
  done
done
grep '^{' $O/micro.log
