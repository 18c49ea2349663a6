#!/bin/bash
# Round 5 batch 27: cell-grid scan with node records stored in cell order (one LDS read per
# candidate) and the grid's bounding box taken during staging (no chunk boxes on the cell path).
# in-tree (2-D cells) vs alt_so/prev (the committed 2-D cell version); alt_so/c3 = in-tree + 3-D
# cells. Tests of both, phase clocks, interleaved headline fp32 x3 (prev vs cur), config #5 fp16 x2
# (cur vs c3), 3-D kernel trace of c3. Output: gpurun_out/${TAG:-r5b27}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b27}
mkdir -p $O
P=$GRAFT_REPO_ROOT/alt_so/prev/_C.so
X=$GRAFT_REPO_ROOT/alt_so/c3/_C.so
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
T="tests/test_gpu_nd.py tests/test_gpu_forward.py tests/test_gpu_runtime.py tests/test_gpu_small.py"
timeout -k 10 400 python -u -m pytest $T -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_cur.log 2>&1
rc=$?; tail -1 $O/tests_cur.log; if [ $rc -ne 0 ]; then echo "STOP cur tests"; exit $rc; fi
MACBF_EXT=$X timeout -k 10 400 python -u -m pytest tests/test_gpu_nd.py tests/test_gpu_forward.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_c3.log 2>&1
rc=$?; tail -1 $O/tests_c3.log; if [ $rc -ne 0 ]; then echo "STOP c3 tests"; exit $rc; fi
timeout -k 10 200 python scripts/stamps_scan.py > $O/stamps_cur_2d.log 2>&1 && tail -14 $O/stamps_cur_2d.log | head -7 || { echo STOP stamps; exit 1; }
MACBF_EXT=$X timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_c3_3d.log 2>&1 && tail -14 $O/stamps_c3_3d.log | head -7 || { echo STOP stamps; exit 1; }
for rep in 1 2 3; do
  MACBF_EXT=$P timeout -k 10 200 python bench.py > $O/prev_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  timeout -k 10 200 python bench.py > $O/cur_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "fp32 $rep prev $(ms $O/prev_fp32_$rep.log) cur $(ms $O/cur_fp32_$rep.log)"
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/c3_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 fp16 $rep cur $(ms $O/cur_cfg5_$rep.log) c3 $(ms $O/c3_cfg5_$rep.log)"
done
cd /tmp && export TMPDIR=/tmp
MACBF_EXT=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --dim 3 --num_obstacles 8 --dtype fp16 > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
cp $(find $O/prof_c3 -name "*kernel_stats.csv" | head -1) $O/kernel_stats_cfg5_c3.csv
echo "c3 $(python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_cfg5_c3.csv 3 | grep -i scan_kernel)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cur -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $O/prof_cur.log 2>&1 || { tail -5 $O/prof_cur.log; exit 1; }
cp $(find $O/prof_cur -name "*kernel_stats.csv" | head -1) $O/kernel_stats_headline_cur.csv
echo "cur $(python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_headline_cur.csv 8 | grep -i scan_kernel)"
