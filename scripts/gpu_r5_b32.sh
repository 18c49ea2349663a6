#!/bin/bash
# Round 5 batch 32: alt_so/rtf = cell-row table walked only over the agent's rows + cell records
# carrying the speed (SCAN_CELL_VZ), vs in-tree (rows advanced inside the candidate loop). Tests,
# phase clocks, interleaved headline fp32 x3, bf16 x1, config #5 fp16 x2.
# Output: gpurun_out/${TAG:-r5b32}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b32}
mkdir -p $O
X=$GRAFT_REPO_ROOT/alt_so/rtf/_C.so
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
T="tests/test_gpu_nd.py tests/test_gpu_forward.py tests/test_gpu_runtime.py tests/test_gpu_small.py tests/test_gpu_fp32.py"
MACBF_EXT=$X timeout -k 10 400 python -u -m pytest $T -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_rtf.log 2>&1
rc=$?; tail -1 $O/tests_rtf.log; if [ $rc -ne 0 ]; then echo "STOP rtf tests"; exit $rc; fi
MACBF_EXT=$X timeout -k 10 200 python scripts/stamps_scan.py > $O/stamps_rtf_2d.log 2>&1 && tail -14 $O/stamps_rtf_2d.log | head -7 || { echo STOP stamps; exit 1; }
MACBF_EXT=$X timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_rtf_3d.log 2>&1 && tail -14 $O/stamps_rtf_3d.log | head -7 || { echo STOP stamps; exit 1; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/cur_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 200 python bench.py > $O/rtf_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "fp32 $rep cur $(ms $O/cur_fp32_$rep.log) rtf $(ms $O/rtf_fp32_$rep.log)"
done
timeout -k 10 200 python bench.py --dtype bf16 > $O/cur_bf16.log 2>&1 || { echo STOP; exit 1; }
MACBF_EXT=$X timeout -k 10 200 python bench.py --dtype bf16 > $O/rtf_bf16.log 2>&1 || { echo STOP; exit 1; }
echo "bf16 cur $(ms $O/cur_bf16.log) rtf $(ms $O/rtf_bf16.log)"
for rep in 1 2; do
  timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cur_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/rtf_cfg5_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "cfg5 fp16 $rep cur $(ms $O/cur_cfg5_$rep.log) rtf $(ms $O/rtf_cfg5_$rep.log)"
done
cd /tmp && export TMPDIR=/tmp
MACBF_EXT=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --dim 3 --num_obstacles 8 --dtype fp16 > $O/prof_cfg5.log 2>&1 || { tail -5 $O/prof_cfg5.log; exit 1; }
cp $(find $O/prof_cfg5 -name "*kernel_stats.csv" | head -1) $O/kernel_stats_cfg5_rtf.csv
echo "cfg5 $(python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_cfg5_rtf.csv 3 | grep -i scan_kernel)"
MACBF_EXT=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_hl -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $O/prof_hl.log 2>&1 || { tail -5 $O/prof_hl.log; exit 1; }
cp $(find $O/prof_hl -name "*kernel_stats.csv" | head -1) $O/kernel_stats_headline_rtf.csv
echo "headline $(python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_headline_rtf.csv 8 | grep -i scan_kernel)"
