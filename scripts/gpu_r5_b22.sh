#!/bin/bash
# Round 5 batch 22 (measurements): kernel traces of (a) the headline with the sampler inline
# (MACBF_PREFETCH=0: is the CBF backward stretched by the overlapped sampler?) and (b) config #5
# fp16 (3-D scan time per call). Output: gpurun_out/${TAG:-r5b22}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b22}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
MACBF_PREFETCH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_pf0 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $O/prof_pf0.log 2>&1 || { tail -5 $O/prof_pf0.log; exit 1; }
cp $(find $O/prof_pf0 -name "*kernel_stats.csv" | head -1) $O/kernel_stats_pf0.csv
cp $(find $O/prof_pf0 -name "*kernel_trace.csv" | head -1) $O/kernel_trace_pf0.csv
python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_pf0.csv 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --dim 3 --num_obstacles 8 --dtype fp16 > $O/prof_cfg5.log 2>&1 || { tail -5 $O/prof_cfg5.log; exit 1; }
cp $(find $O/prof_cfg5 -name "*kernel_stats.csv" | head -1) $O/kernel_stats_cfg5_fp16.csv
python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_cfg5_fp16.csv 12
