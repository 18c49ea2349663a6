#!/bin/bash
# Kernel traces of the latency-bound configurations: the DP=8 per-rank slice of config #3
# (8 envs x 1024 agents) and BASELINE config #2 (32 agents x 1 env), plus their benches with
# per-phase timings. Output: gpurun_out/${TAG:-slices}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-slices}
mkdir -p $O
timeout -k 10 200 python bench.py --envs 8 --steps 20 --warmup 5 --phases > $O/slice8.log 2>&1 || { tail -5 $O/slice8.log; exit 1; }
timeout -k 10 200 python bench.py --agents 32 --envs 1 --steps 40 --warmup 10 --phases > $O/cfg2.log 2>&1 || { tail -5 $O/cfg2.log; exit 1; }
for f in slice8 cfg2; do python -c "import json; d=json.loads(open('$O/$f.log').read().strip().split(chr(10))[-1]); print('$f', round(d['ms_per_step'],3), round(d['value']/1e6,3), d.get('phases_ms'))"; done
TAG=${TAG:-slices}/p8 STEPS=6 ARGS="--envs 8" bash scripts/gpu_prof.sh > /dev/null || exit 1
TAG=${TAG:-slices}/p2 STEPS=10 ARGS="--agents 32 --envs 1" bash scripts/gpu_prof.sh > /dev/null || exit 1
python scripts/iter_kernels.py $O/p8/kernel_trace.csv > $O/p8/iter.txt; head -30 $O/p8/iter.txt
python scripts/iter_kernels.py $O/p2/kernel_trace.csv > $O/p2/iter.txt; head -30 $O/p2/iter.txt
