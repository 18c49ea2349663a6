# Run selected GPU tests against each prebuilt variant (scripts/build_variants.sh) by swapping
# the in-tree extension, then restore it. usage: bash scripts/gpu_variants_tests.sh "TESTS" v1 v2 ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1; shift
SO=$(ls macbf_gnn_amd/_C*.so)
cp $SO /tmp/_C_orig.so
for v in "$@"; do
  cp build/variants/$v/_C.so $SO
  timeout -k 10 300 python -u -m pytest $T -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/vt_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc"; tail -1 gpurun_out/vt_$v.log
  if [ $rc -gt 1 ]; then cp /tmp/_C_orig.so $SO; exit $rc; fi
done
cp /tmp/_C_orig.so $SO
