#!/bin/bash
# Round 5 batch 30: cell-grid candidate walk. in-tree = trimmed row segments (one contiguous range
# per cell row, rows cut to the sphere, candidates dealt to the agent's lanes round-robin);
# alt_so/gap = per-lane cells with per-cell distance skips; alt_so/nogap = batch 29's per-lane cells.
# Tests of all three, phase clocks of in-tree, interleaved headline fp32 x2 and config #5 fp16 x2.
# Output: gpurun_out/${TAG:-r5b30}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b30}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
T="tests/test_gpu_nd.py tests/test_gpu_forward.py tests/test_gpu_runtime.py tests/test_gpu_small.py"
timeout -k 10 400 python -u -m pytest $T -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_cur.log 2>&1
rc=$?; tail -1 $O/tests_cur.log; if [ $rc -ne 0 ]; then echo "STOP cur tests"; exit $rc; fi
MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/gap/_C.so timeout -k 10 300 python -u -m pytest tests/test_gpu_nd.py tests/test_gpu_forward.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_gap.log 2>&1
rc=$?; tail -1 $O/tests_gap.log; if [ $rc -ne 0 ]; then echo "STOP gap tests"; exit $rc; fi
timeout -k 10 200 python scripts/stamps_scan.py > $O/stamps_cur_2d.log 2>&1 && tail -14 $O/stamps_cur_2d.log | head -13 || { echo STOP stamps; exit 1; }
timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_cur_3d.log 2>&1 && tail -14 $O/stamps_cur_3d.log | head -13 || { echo STOP stamps; exit 1; }
for rep in 1 2; do
  line="fp32 $rep"
  for v in nogap gap cur; do
    if [ $v = cur ]; then E=; else E=$GRAFT_REPO_ROOT/alt_so/$v/_C.so; fi
    MACBF_EXT=$E timeout -k 10 200 python bench.py > $O/${v}_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
    line="$line $v $(ms $O/${v}_fp32_$rep.log)"
  done
  echo "$line"
done
for rep in 1 2; do
  line="cfg5 fp16 $rep"
  for v in nogap gap cur; do
    if [ $v = cur ]; then E=; else E=$GRAFT_REPO_ROOT/alt_so/$v/_C.so; fi
    MACBF_EXT=$E timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/${v}_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
    line="$line $v $(ms $O/${v}_cfg5_$rep.log)"
  done
  echo "$line"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --dim 3 --num_obstacles 8 --dtype fp16 > $O/prof_cfg5.log 2>&1 || { tail -5 $O/prof_cfg5.log; exit 1; }
cp $(find $O/prof_cfg5 -name "*kernel_stats.csv" | head -1) $O/kernel_stats_cfg5_cur.csv
echo "cfg5 $(python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_cfg5_cur.csv 3 | grep -i scan_kernel)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_hl -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $O/prof_hl.log 2>&1 || { tail -5 $O/prof_hl.log; exit 1; }
cp $(find $O/prof_hl -name "*kernel_stats.csv" | head -1) $O/kernel_stats_headline_cur.csv
echo "headline $(python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_headline_cur.csv 8 | grep -i scan_kernel)"
