#!/bin/bash
# Round 5 batch 14: scan block-level imbalance (phase clocks: the median wave waits ~24 k cycles at
# the block's count barrier). Variants: per-wave count atomics without the barrier
# (alt_so/wavatom), 512-thread blocks = two blocks per CU (alt_so/bs512). Tests per variant, kernel
# traces, interleaved headline fp32 x2 and config #5 fp16 x1. Output: gpurun_out/${TAG:-r5b14}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b14}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
for v in wavatom bs512; do
  MACBF_EXT=alt_so/$v/_C.so timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_runtime.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; tail -1 $O/tests_$v.log; if [ $rc -ne 0 ]; then echo "STOP $v tests"; exit $rc; fi
done
cd /tmp && export TMPDIR=/tmp
for v in cur wavatom bs512; do
  if [ $v != cur ]; then export MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$v/_C.so; else unset MACBF_EXT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  cp $(find $O/prof_$v -name "*kernel_stats.csv" | head -1) $O/kernel_stats_$v.csv
  echo "$v: $(python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_$v.csv 10 | grep -i scan_kernel)"
done
unset MACBF_EXT
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in cur wavatom bs512; do
    if [ $v != cur ]; then E="MACBF_EXT=alt_so/$v/_C.so"; else E=""; fi
    env $E timeout -k 10 200 python bench.py > $O/${v}_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  done
  echo "fp32 $rep cur $(ms $O/cur_fp32_$rep.log) wavatom $(ms $O/wavatom_fp32_$rep.log) bs512 $(ms $O/bs512_fp32_$rep.log)"
done
for v in cur wavatom bs512; do
  if [ $v != cur ]; then E="MACBF_EXT=alt_so/$v/_C.so"; else E=""; fi
  env $E timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/${v}_cfg5.log 2>&1 || { echo STOP; exit 1; }
done
echo "cfg5 cur $(ms $O/cur_cfg5.log) wavatom $(ms $O/wavatom_cfg5.log) bs512 $(ms $O/bs512_cfg5.log)"
