#!/bin/bash
# Round 5 batch 2: GPU suite (DP split all-reduce, node16 self-check, tie gates), then kernel traces
# of the latency-bound configurations: config #2 (32 x 1, bf16) and the 8-env slice (fp32).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -4 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
TAG=${TAG:-r5b2}/cfg2 STEPS=30 ARGS="--agents 32 --envs 1 --dtype bf16 --phases" bash scripts/gpu_prof.sh > $O/cfg2_summary.txt 2>&1 && head -16 $O/cfg2_summary.txt
TAG=${TAG:-r5b2}/slice8 STEPS=20 ARGS="--agents 1024 --envs 8 --phases" bash scripts/gpu_prof.sh > $O/slice8_summary.txt 2>&1 && head -16 $O/slice8_summary.txt
