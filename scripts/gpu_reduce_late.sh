# Edge->node reduction split in time (MACBF_REDUCE_LATE=k: the last k steps' dS before the BPTT,
# the rest on the aux stream during the first BPTT steps) vs one reduction (default 0): interleaved
# headline benches (20 steps). Output: gpurun_out/rlate
cd $GRAFT_REPO_ROOT
O=gpurun_out/rlate
mkdir -p $O
for rep in 1 2; do
  for v in 0 2 4; do
    MACBF_REDUCE_LATE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_${v}_$rep.log 2>&1 || { tail -5 $O/b_${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${v}_$rep.log').read().strip().split(chr(10))[-1]); print('reduce_late $v', round(d['ms_per_step'],3))"
  done
done
