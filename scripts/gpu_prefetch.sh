# Scenario prefetch on a side stream (default) vs in-line sampling (MACBF_PREFETCH=0): interleaved
# headline bench A/B + one kernel trace of each. Output: gpurun_out/pref
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/pref
mkdir -p $O
for rep in 1 2; do
  for v in 1 0; do
    MACBF_PREFETCH=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_${v}_$rep.log 2>&1 || { tail -5 $O/b_${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${v}_$rep.log').read().strip().split(chr(10))[-1]); print('prefetch $v', round(d['ms_per_step'],3))"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  MACBF_PREFETCH=$v timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $O/prof$v.log 2>&1 || exit 1
done
