#!/bin/bash
# rocprofv3 kernel trace + stats of a short headline bench (ARGS: extra bench.py flags).
# Output: gpurun_out/${TAG:-prof}/kernel_stats.csv (+ the per-dispatch trace)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps ${STEPS:-4} --warmup 2 $ARGS > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
cp $(find $O/prof -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv
python scripts/kstats.py $O/kernel_stats.csv 45
