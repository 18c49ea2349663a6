#!/bin/bash
# Round 5 batch 25: cell-grid scan in 2-D and 3-D (alt_so/cell23, -DSCAN_CELL2=1 -DSCAN_CELL3=1):
# scan / 3-D / runtime / small-scene tests with the variant, 2-D and 3-D phase clocks, interleaved
# headline fp32 x3, bf16 x1, config #5 fp16 x2, kernel traces. Output: gpurun_out/${TAG:-r5b25}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b25}
mkdir -p $O
ALT=${ALT:-cell23}
X=$GRAFT_REPO_ROOT/alt_so/$ALT/_C.so
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
MACBF_EXT=$X timeout -k 10 400 python -u -m pytest tests/test_gpu_nd.py tests/test_gpu_forward.py tests/test_gpu_runtime.py tests/test_gpu_small.py tests/test_gpu_fp32.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_alt.log 2>&1
rc=$?; tail -1 $O/tests_alt.log; if [ $rc -ne 0 ]; then echo "STOP alt tests"; exit $rc; fi
MACBF_EXT=$X timeout -k 10 200 python scripts/stamps_scan.py > $O/stamps_alt_2d.log 2>&1 && tail -14 $O/stamps_alt_2d.log | head -7 || { echo STOP stamps; exit 1; }
MACBF_EXT=$X timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_alt_3d.log 2>&1 && tail -14 $O/stamps_alt_3d.log | head -7 || { echo STOP stamps; exit 1; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/cur_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 200 python bench.py > $O/alt_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "fp32 $rep cur $(ms $O/cur_fp32_$rep.log) alt $(ms $O/alt_fp32_$rep.log)"
done
timeout -k 10 200 python bench.py --dtype bf16 > $O/cur_bf16.log 2>&1 || { echo STOP; exit 1; }
MACBF_EXT=$X timeout -k 10 200 python bench.py --dtype bf16 > $O/alt_bf16.log 2>&1 || { echo STOP; exit 1; }
echo "bf16 cur $(ms $O/cur_bf16.log) alt $(ms $O/alt_bf16.log)"
for rep in 1 2; do
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/alt_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 fp16 $rep cur $(ms $O/cur_cfg5_$rep.log) alt $(ms $O/alt_cfg5_$rep.log)"
done
cd /tmp && export TMPDIR=/tmp
MACBF_EXT=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_alt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $O/prof_alt.log 2>&1 || { tail -5 $O/prof_alt.log; exit 1; }
cp $(find $O/prof_alt -name "*kernel_stats.csv" | head -1) $O/kernel_stats_headline_alt.csv
python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_headline_alt.csv 8 | grep -i scan || true
