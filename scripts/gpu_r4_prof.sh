#!/bin/bash
# Profiles of the current build: SOL table of the headline (two PMC passes over bench.py) and kernel
# traces (--kernel-trace --stats) of the headline, the 8-env slice, bf16 and config #5 fp16.
# Output: gpurun_out/${TAG:-r4p}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r4p}
mkdir -p $O
stop() { echo "STOP: $1 rc=$2"; exit $2; }
TAG=${TAG:-r4p}/sol bash scripts/gpu_sol.sh > $O/sol.log 2>&1 || stop sol $?
head -12 $O/sol.log
cd /tmp && export TMPDIR=/tmp
export MACBF_SELFCHECK=0
for cfg in "headline:" "slice8:--envs 8" "bf16:--dtype bf16" "fp16cfg5:--dim 3 --num_obstacles 8 --dtype fp16"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_$name -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 $args > $GRAFT_REPO_ROOT/$O/trace_$name.log 2>&1 || stop trace_$name $?
  grep '^{' $GRAFT_REPO_ROOT/$O/trace_$name.log | cut -c1-120
done
