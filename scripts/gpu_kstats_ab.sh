# Per-kernel A/B under rocprofv3 --kernel-trace --stats: bench.py --steps 3 for the in-tree
# build and each variant of $VARIANTS (MACBF_EXT), summary of the kernels matching $KPAT
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-kab}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in base $VARIANTS; do
  if [ $v = base ]; then unset MACBF_EXT; else export MACBF_EXT=$GRAFT_REPO_ROOT/build/variants/$v/_C.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 ${BARGS} > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
done
unset MACBF_EXT
cd $GRAFT_REPO_ROOT
for v in base $VARIANTS; do
  f=$(ls $O/$v/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls $O/$v/run_kernel_stats.csv)
  python -c "
import csv, re
for r in csv.DictReader(open('$f')):
    if re.search('${KPAT:-.}', r['Name']): print('$v', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
done
