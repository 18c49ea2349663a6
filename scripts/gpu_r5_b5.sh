#!/bin/bash
# Round 5 batch 5: GPU suite; config #2 with the per-T backward graphs on / off (interleaved);
# fixed-horizon headline (fp32 / bf16 benches + kernel trace); node16 phase clocks at the headline.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b5}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -4 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
for rep in 1 2; do
  for gr in 1 0; do
    for dt in bf16 fp32; do
      MACBF_BWD_GRAPH=$gr timeout -k 10 200 python bench.py --agents 32 --envs 1 --steps 30 --warmup 5 --dtype $dt > $O/cfg2_${dt}_g${gr}_$rep.log 2>&1 || { echo STOP; tail -3 $O/cfg2_${dt}_g${gr}_$rep.log; exit 1; }
      echo "cfg2 $dt graph=$gr $rep $(ms $O/cfg2_${dt}_g${gr}_$rep.log)"
    done
  done
done
for dt in fp32 bf16; do
  timeout -k 10 300 python bench.py --no_early_stop --dtype $dt > $O/fixedT_$dt.log 2>&1 || { echo STOP; tail -3 $O/fixedT_$dt.log; exit 1; }
  echo "fixedT $dt $(ms $O/fixedT_$dt.log)"
done
timeout -k 10 200 python scripts/stamps_node.py --node16 --envs 64 > $O/stamps_node16.log 2>&1 && tail -14 $O/stamps_node16.log
TAG=${TAG:-r5b5}/fixedT STEPS=4 ARGS="--no_early_stop" bash scripts/gpu_prof.sh > $O/fixedT_summary.txt 2>&1 && head -8 $O/fixedT_summary.txt
