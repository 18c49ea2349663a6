# Time the CBF training kernel for each prebuilt ablation variant (scripts/build_variants.sh cbf).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 300 python scripts/micro_cbf.py --so build/variants/$v/_C.so --tag $v >> gpurun_out/cbf_ablation.log 2>&1
  rc=$?; tail -1 gpurun_out/cbf_ablation.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
