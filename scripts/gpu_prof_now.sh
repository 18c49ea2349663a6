#!/bin/bash
# Headline kernel trace (rocprofv3 --kernel-trace --stats, 6 timed iterations) + the 8-env slice
# (DP 8 of config #3 as stated) and config #2 benches with per-phase timings.
# Output: gpurun_out/${TAG:-prof}
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-prof}
mkdir -p $O
timeout -k 10 300 python bench.py --envs 8 --steps 20 --warmup 5 --phases > $O/slice8.log 2>&1 || { tail -5 $O/slice8.log; exit 1; }
timeout -k 10 300 python bench.py --agents 32 --envs 1 --steps 30 --warmup 5 --phases > $O/cfg2.log 2>&1 || { tail -5 $O/cfg2.log; exit 1; }
for f in slice8 cfg2; do python -c "import json; d=json.loads(open('$O/$f.log').read().strip().split(chr(10))[-1]); print('$f', round(d['ms_per_step'],3), round(d['value']/1e6,3), d.get('phases_ms'))"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
python scripts/kstats.py $O/kernel_stats.csv 22
