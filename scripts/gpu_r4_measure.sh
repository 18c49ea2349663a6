#!/bin/bash
# Round-4 measurement pass on one box: SOL table of the headline (two PMC passes over bench.py),
# PMC baselines of the profiler test (both workloads, re-recorded), kernel traces of the headline and
# of the 8-env strong-scaling slice, node16 phase clocks. Output: gpurun_out/${TAG:-r4m}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r4m}
mkdir -p $O
stop() { echo "STOP: $1 rc=$2"; exit $2; }
TAG=${TAG:-r4m}/sol bash scripts/gpu_sol.sh > $O/sol.log 2>&1 || stop sol $?
tail -30 $O/sol.log
MACBF_PMC_RECORD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_profiler.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pmc_record.log 2>&1
rc=$?; tail -5 $O/pmc_record.log; [ $rc -le 1 ] || stop pmc $rc
cd /tmp && export TMPDIR=/tmp
export MACBF_SELFCHECK=0
for cfg in "headline:" "slice8:--envs 8" "bf16:--dtype bf16"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_$name -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 $args > $GRAFT_REPO_ROOT/$O/trace_$name.log 2>&1 || stop trace_$name $?
  grep '^{' $GRAFT_REPO_ROOT/$O/trace_$name.log | cut -c1-160
done
cd $GRAFT_REPO_ROOT
unset MACBF_SELFCHECK
timeout -k 10 200 python -u scripts/stamps_node.py --node16 --envs 64 > $O/stamps16.log 2>&1 || stop stamps $?
tail -20 $O/stamps16.log
