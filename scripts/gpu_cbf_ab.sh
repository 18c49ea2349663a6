# Interleaved A/B of CBF kernel variants (scripts/build_variants.sh cbf_x3 ...) with
# scripts/micro_cbf_dedup.py: VARIANTS="base name ..." (base = in-tree build). Output: gpurun_out/${TAG:-cbfab}
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cbfab}
mkdir -p $O
for rep in 1 2; do
  for v in $VARIANTS; do
    if [ $v = base ]; then unset MACBF_EXT; else export MACBF_EXT=$GRAFT_REPO_ROOT/build/variants/$v/_C.so; fi
    timeout -k 10 200 python scripts/micro_cbf_dedup.py --dtype ${DTYPE:-fp32} --tag $v >> $O/micro_cbf.log 2>&1 || { tail -5 $O/micro_cbf.log; exit 1; }
  done
done
unset MACBF_EXT
grep '^{' $O/micro_cbf.log
