#!/bin/bash
# Round 5 batch 26: 3-D cell-grid scan (alt_so/cell3, -DSCAN_CELL3=1; 2-D cells are the default
# now) vs the 3-D chunk culling: config #5 fp16 x3 / fp32 x1 interleaved, kernel traces of both.
# Output: gpurun_out/${TAG:-r5b26}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b26}
mkdir -p $O
X=$GRAFT_REPO_ROOT/alt_so/${ALT:-cell3}/_C.so
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_nd.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_cur.log 2>&1
rc=$?; tail -1 $O/tests_cur.log; if [ $rc -ne 0 ]; then echo "STOP cur tests"; exit $rc; fi
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/alt_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 fp16 $rep cur $(ms $O/cur_cfg5_$rep.log) alt $(ms $O/alt_cfg5_$rep.log)"
done
timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 > $O/cur_cfg5_fp32.log 2>&1 || { echo STOP; exit 1; }
MACBF_EXT=$X timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 > $O/alt_cfg5_fp32.log 2>&1 || { echo STOP; exit 1; }
echo "cfg5 fp32 cur $(ms $O/cur_cfg5_fp32.log) alt $(ms $O/alt_cfg5_fp32.log)"
cd /tmp && export TMPDIR=/tmp
for v in cur alt; do
  if [ $v = alt ]; then export MACBF_EXT=$X; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --dim 3 --num_obstacles 8 --dtype fp16 > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  cp $(find $O/prof_$v -name "*kernel_stats.csv" | head -1) $O/kernel_stats_cfg5_$v.csv
  echo "$v $(python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_cfg5_$v.csv 3 | grep -i scan_kernel)"
done
