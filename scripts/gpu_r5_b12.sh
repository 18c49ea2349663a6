#!/bin/bash
# Round 5 batch 12: kNN scan without the per-chunk threshold / all-danger updates when no lane of the
# wave changed (alt_so/thrskip, -DSCAN_THR_SKIP=1): scan / 3-D / runtime tests with the variant,
# kernel traces of the headline for both builds, interleaved A/B: headline fp32 x3, config #5
# fp16 x2. Output: gpurun_out/${TAG:-r5b12}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b12}
mkdir -p $O
ALT=${ALT:-thrskip}
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
MACBF_EXT=alt_so/$ALT/_C.so timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_nd.py tests/test_gpu_runtime.py tests/test_gpu_small.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/alt_tests.log 2>&1
rc=$?; tail -2 $O/alt_tests.log; if [ $rc -ne 0 ]; then echo "STOP alt tests"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
for v in cur alt; do
  if [ $v = alt ]; then export MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$ALT/_C.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  cp $(find $O/prof_$v -name "*kernel_stats.csv" | head -1) $O/kernel_stats_$v.csv
  python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_$v.csv 8 | grep -i "scan" || true
done
unset MACBF_EXT
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/cur_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=alt_so/$ALT/_C.so timeout -k 10 200 python bench.py > $O/alt_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "fp32 $rep cur $(ms $O/cur_fp32_$rep.log) alt $(ms $O/alt_fp32_$rep.log)"
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=alt_so/$ALT/_C.so timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/alt_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 $rep cur $(ms $O/cur_cfg5_$rep.log) alt $(ms $O/alt_cfg5_$rep.log)"
done
