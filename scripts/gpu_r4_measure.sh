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
for cfg in "headline:" "slice8:--envs 8" "bf16:--dtype bf16" "fp16cfg5:--dim 3 --num_obstacles 8 --dtype fp16"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_$name -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 $args > $GRAFT_REPO_ROOT/$O/trace_$name.log 2>&1 || stop trace_$name $?
  grep '^{' $GRAFT_REPO_ROOT/$O/trace_$name.log | cut -c1-160
done
# the same 1-pass configs with the 32x32x16 backward kernels (per-kernel A/B)
export MACBF_CBF16=0 MACBF_EB16=0 MACBF_NODE16=0
for cfg in "bf16_k32:--dtype bf16" "fp16cfg5_k32:--dim 3 --num_obstacles 8 --dtype fp16"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_$name -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 $args > $GRAFT_REPO_ROOT/$O/trace_$name.log 2>&1 || stop trace_$name $?
  grep '^{' $GRAFT_REPO_ROOT/$O/trace_$name.log | cut -c1-160
done
unset MACBF_CBF16 MACBF_EB16 MACBF_NODE16
cd $GRAFT_REPO_ROOT
unset MACBF_SELFCHECK
# fp32 headline: sched barriers on (default) / off (no-barrier builds), interleaved
for rep in 1 2; do
  for v in default cbf_nobar ctrl_nobar; do
    if [ $v = default ]; then E=X=1; else E=MACBF_EXT=alt_so/$v/_C.so; fi
    env $E timeout -k 10 300 python bench.py > $O/fp32_${v}_${rep}.log 2>&1 || stop fp32_$v $?
    echo "fp32 $v $rep: $(grep '^{' $O/fp32_${v}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms")')"
  done
done
