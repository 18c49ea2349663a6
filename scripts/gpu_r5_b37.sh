#!/bin/bash
# Round 5 batch 37: config #5 fp16 kernel trace on the final build (3-D scan per call).
# Output: gpurun_out/${TAG:-r5b37}/
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b37}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --dim 3 --num_obstacles 8 --dtype fp16 > $O/prof_cfg5.log 2>&1 || { tail -5 $O/prof_cfg5.log; exit 1; }
cp $(find $O/prof_cfg5 -name "*kernel_stats.csv" | head -1) $O/kernel_stats_cfg5_fp16.csv
python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_cfg5_fp16.csv 8
