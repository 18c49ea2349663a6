# LDS-DMA weight staging (block_copy16 -> global_load_lds): full GPU suite, then interleaved A/B
# against the register-staged copy (build/variants/oldcopy: ctrl_x3 with -DMB_GLDS_COPY=0) with
# the per-step micro-benchmark (headline and 32 x 1) and the config #2 bench. Output: gpurun_out/glds
cd $GRAFT_REPO_ROOT
O=gpurun_out/glds
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base oldcopy; do
    if [ $v = base ]; then SO=""; unset MACBF_EXT; else SO="--so build/variants/$v/_C.so"; export MACBF_EXT=$GRAFT_REPO_ROOT/build/variants/$v/_C.so; fi
    timeout -k 10 300 python scripts/micro_step.py $SO --tag ${v}_$rep >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
    timeout -k 10 300 python scripts/micro_step.py $SO --agents 32 --envs 1 --tag ${v}_32x1_$rep >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
    timeout -k 10 300 python bench.py --agents 32 --envs 1 --steps 30 --warmup 5 > $O/cfg2_${v}_$rep.log 2>&1 || { tail -5 $O/cfg2_${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/cfg2_${v}_$rep.log').read().strip().split(chr(10))[-1]); print('cfg2 $v', round(d['ms_per_step'],3))"
  done
done
unset MACBF_EXT
grep '^{' $O/micro.log
