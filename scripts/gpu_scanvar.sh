# scan variants (scripts/build_variants.sh scan ...): per-step micro-benchmarks, interleaved
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-scanvar}
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python scripts/micro_step.py --dtype fp32 --tag base >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
  for v in ${VARIANTS}; do
    timeout -k 10 200 python scripts/micro_step.py --dtype fp32 --so build/variants/$v/_C.so --tag $v >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
  done
done
grep '^{' $O/micro.log | python -c "import sys,json; [print(d['tag'], d['scan'], d['scan_nosort'], d['scan_noprev'], d['scan_safeonly']) for d in map(json.loads, sys.stdin)]"
