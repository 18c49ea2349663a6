# x3 (fp32) ablation sweep: per-step kernel micro-benchmarks (controller) and bench phases (CBF)
# for variants built by scripts/build_variants.sh ctrl_x3 / cbf_x3. Output: gpurun_out/${TAG:-abl}
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abl}
mkdir -p $O
timeout -k 10 200 python scripts/micro_step.py --dtype fp32 --tag base > $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
for v in ${CTRL_VARIANTS:-x3_nostage x3_nos1 x3_nos2 x3_noslab}; do
  timeout -k 10 200 python scripts/micro_step.py --dtype fp32 --so build/variants/$v/_C.so --tag $v >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
done
grep '^{' $O/micro.log
for v in base ${CBF_VARIANTS:-cx3_nostage cx3_nostmma cx3_noststore cx3_noload}; do
  if [ $v = base ]; then unset MACBF_EXT; else export MACBF_EXT=$GRAFT_REPO_ROOT/build/variants/$v/_C.so; fi
  timeout -k 10 200 python scripts/micro_cbf_dedup.py --dtype fp32 --tag $v >> $O/micro_cbf.log 2>&1 || { tail -5 $O/micro_cbf.log; exit 1; }
done
unset MACBF_EXT
grep '^{' $O/micro_cbf.log
