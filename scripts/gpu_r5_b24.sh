#!/bin/bash
# Round 5 batch 24: 3-D scan over a per-env cell grid around each agent (alt_so/cell3,
# -DSCAN_CELL3=1). 3-D / scan / runtime tests (in-tree and variant; the new 1,024-agent 3-D
# temporal-bound test), 3-D phase clocks, interleaved config #5 fp16 x2 + fp32 x1, kernel trace.
# Output: gpurun_out/${TAG:-r5b24}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b24}
mkdir -p $O
ALT=${ALT:-cell3}
X=$GRAFT_REPO_ROOT/alt_so/$ALT/_C.so
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_nd.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_cur.log 2>&1
rc=$?; tail -1 $O/tests_cur.log; if [ $rc -ne 0 ]; then echo "STOP cur tests"; exit $rc; fi
MACBF_EXT=$X timeout -k 10 400 python -u -m pytest tests/test_gpu_nd.py tests/test_gpu_forward.py tests/test_gpu_runtime.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_alt.log 2>&1
rc=$?; tail -1 $O/tests_alt.log; if [ $rc -ne 0 ]; then echo "STOP alt tests"; exit $rc; fi
MACBF_EXT=$X timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_alt_3d.log 2>&1 && tail -14 $O/stamps_alt_3d.log | head -8 || { echo STOP stamps; exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/alt_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 fp16 $rep cur $(ms $O/cur_cfg5_$rep.log) alt $(ms $O/alt_cfg5_$rep.log)"
done
timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 > $O/cur_cfg5_fp32.log 2>&1 || { echo STOP; exit 1; }
MACBF_EXT=$X timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 > $O/alt_cfg5_fp32.log 2>&1 || { echo STOP; exit 1; }
echo "cfg5 fp32 cur $(ms $O/cur_cfg5_fp32.log) alt $(ms $O/alt_cfg5_fp32.log)"
cd /tmp && export TMPDIR=/tmp
MACBF_EXT=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_alt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --dim 3 --num_obstacles 8 --dtype fp16 > $O/prof_alt.log 2>&1 || { tail -5 $O/prof_alt.log; exit 1; }
cp $(find $O/prof_alt -name "*kernel_stats.csv" | head -1) $O/kernel_stats_cfg5_alt.csv
python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_cfg5_alt.csv 4
