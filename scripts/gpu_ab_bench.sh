# Interleaved bench A/B: in-tree build vs variant $V (MACBF_EXT), both dtypes, 3 rounds each
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abb}
mkdir -p $O
for rep in 1 2 3; do
  for dt in ${DTS:-fp32 bf16}; do
    for which in base var; do
      if [ $which = var ]; then export MACBF_EXT=$GRAFT_REPO_ROOT/build/variants/$V/_C.so; else unset MACBF_EXT; fi
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype $dt > $O/b_${dt}_${which}_$rep.log 2>&1 || { tail -5 $O/b_${dt}_${which}_$rep.log; exit 1; }
      python -c "import json; d=json.loads(open('$O/b_${dt}_${which}_$rep.log').read().strip().split(chr(10))[-1]); print('$dt $which $rep', round(d['ms_per_step'],3))"
    done
  done
done
