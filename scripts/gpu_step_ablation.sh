# Time the per-step kernels for each prebuilt variant (scripts/build_variants.sh).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 300 python scripts/micro_step.py --so build/variants/$v/_C.so --tag $v >> gpurun_out/step_ablation.log 2>&1
  rc=$?; tail -1 gpurun_out/step_ablation.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
