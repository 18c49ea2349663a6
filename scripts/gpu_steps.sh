#!/bin/bash
# Round-6 GPU driver: one parameterised script instead of a batch script per experiment. Runs the
# named steps in order, each under its own time limit; the first failure (or fault / timeout) ends
# the call. Output: gpurun_out/${TAG:-r6}/.
#
#   STEPS="tests smoke bench slice cfg2 prof_slice prof neg" TAG=r6a bash scripts/gpu_steps.sh
#
# tests        full GPU suite (pytest -m gpu)                  -> tests.log
# t:<expr>     GPU tests selected by -k <expr>                  -> t_<expr>.log
# smoke        __graft_entry__.smoke()                          -> smoke.log
# bench        bench.py defaults (config #3 as stated)          -> bench.log
# slice        bench.py --envs 8 (the DP=8 per-rank slice)      -> slice.log
# e16 / e32    bench.py --envs 16 / 32 (the DP=4 / DP=2 per-rank work)
# cfg2         bench.py --agents 32 --envs 1 --dtype bf16       -> cfg2.log
# cfg4 / cfg5  config #4 (4096 x 16 fp32) / #5 (3-D + 8 obstacles, fp16)
# bf16         the headline in bf16
# ab:<NAME>    interleaved headline+slice A/B of alt_so/NAME/_C.so vs the in-tree build (REPS; ABARGS
#              replaces the headline's bench args, '+' for spaces: env:ABARGS=--agents+32+--envs+1)
# prof         kernel trace of the headline    -> prof/kernel_stats.csv, prof_summary.txt
# prof_slice   kernel trace of the slice       -> prof_slice/...
# prof_cfg2    kernel trace of config #2 (bf16) -> prof_cfg2/...
# sol / sol_slice / sol_cfg4 / sol_cfg5   two-pass PMC speed-of-light table (scripts/gpu_sol.sh) -> sol_*/sol.md
# configs      every BASELINE config (scripts/gpu_configs.sh)   -> configs/configs.jsonl
# dp:N         N ranks of the bench on this one GPU over gloo (launch / DP rehearsal, strong default)
# neg          scan oracle tests against alt_so/shrink (search box 0.7x): must FAIL -> neg.log
# py:S,ARGS    python scripts/S with comma-separated ARGS (e.g. py:stamps_scan.py,--envs,8) -> py_S.log
# sl:K=V       the slice bench with the env var K=V (A/B of a runtime choice)   -> sl_K_V.log
# e:K=V:STEP   run STEP (a bench step) with the env var K=V        -> K_V_STEP.log
# env:K=V      export K=V for the following steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r6}
mkdir -p $O
B="python -u bench.py"
ms() { grep '^{' $1 | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms", round(d["value"]/1e6,2), "M/s", d["scaling"], d["config"]["global_batch"])'; }
bench() {   # name limit args...
  local n=${PFX:-}$1 t=$2; shift 2
  timeout -k 10 $t $B "$@" > $O/$n.log 2>&1 || { echo "STOP $n rc=$?"; tail -5 $O/$n.log; exit 1; }
  echo "$n: $(ms $O/$n.log)"
}
prof() {    # name args...
  local n=$1; shift
  local P=$GRAFT_REPO_ROOT/$O/$n
  mkdir -p $P
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/raw -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 "$@" > $P/prof.log 2>&1) || { echo "STOP $n"; tail -5 $P/prof.log; exit 1; }
  cp $(find $P/raw -name "*kernel_stats.csv" | head -1) $P/kernel_stats.csv
  cp $(find $P/raw -name "*kernel_trace.csv" | head -1) $P/kernel_trace.csv
  rm -rf $P/raw
  python scripts/kstats.py $P/kernel_stats.csv 30 > $P/summary.txt
  echo "$n: $(grep '^{' $P/prof.log | head -c 200)"
  head -14 $P/summary.txt
}
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1
      rc=$?; tail -4 $O/tests.log
      if [ $rc -ne 0 ]; then echo "STOP tests rc=$rc"; grep -E "^(FAILED|ERROR)" $O/tests.log | head -20; exit $rc; fi ;;
    t:*)
      k=${s#t:}
      timeout -k 10 600 python -u -m pytest tests -v -m gpu -k "$k" -p no:cacheprovider --timeout 240 --timeout-method thread > $O/t_${k//[^a-zA-Z0-9_]/_}.log 2>&1
      rc=$?; tail -3 $O/t_${k//[^a-zA-Z0-9_]/_}.log; if [ $rc -ne 0 ]; then echo "STOP $s rc=$rc"; exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "STOP smoke"; tail -5 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench) bench bench 300 ;;
    slice) bench slice 300 --envs 8 ;;
    e16) bench e16 300 --envs 16 ;;              # the per-rank work of config #3 at DP 4
    e32) bench e32 300 --envs 32 ;;              # ... at DP 2
    cfg2) bench cfg2 300 --agents 32 --envs 1 --steps 30 --dtype bf16 ;;
    cfg2f) bench cfg2f 300 --agents 32 --envs 1 --steps 30 ;;
    cfg4) bench cfg4 300 --agents 4096 --envs 16 ;;
    cfg5) bench cfg5 300 --agents 1024 --envs 64 --dim 3 --num_obstacles 8 --dtype fp16 ;;
    bf16) bench bf16 300 --dtype bf16 ;;
    ab:*)
      alt=alt_so/${s#ab:}/_C.so
      for rep in $(seq 1 ${REPS:-2}); do
        for v in cur alt; do
          for a in "${ABARGS//+/ }" "--envs 8"; do
            tag=${s#ab:}_${v}_$(echo "x$a" | tr -c 'a-zA-Z0-9' _)_$rep
            if [ $v = cur ]; then E=X=1; else E=MACBF_EXT=$alt; fi
            env $E timeout -k 10 300 $B $a > $O/$tag.log 2>&1 || { echo "STOP $tag"; tail -3 $O/$tag.log; exit 1; }
            echo "$tag: $(ms $O/$tag.log)"
          done
        done
      done ;;
    prof) prof prof ;;
    prof_slice) prof prof_slice --envs 8 ;;
    prof_cfg2) prof prof_cfg2 --agents 32 --envs 1 --dtype bf16 ;;
    sol) TAG=${TAG:-r6}/sol ARGS="" bash scripts/gpu_sol.sh > $O/sol.log 2>&1 || { echo "STOP sol"; tail -5 $O/sol.log; exit 1; }; head -30 $O/sol/sol.md ;;
    sol_slice) TAG=${TAG:-r6}/sol_slice ARGS="--envs 8" bash scripts/gpu_sol.sh > $O/sol_slice.log 2>&1 || { echo "STOP sol_slice"; tail -5 $O/sol_slice.log; exit 1; }; head -30 $O/sol_slice/sol.md ;;
    sol_cfg4) TAG=${TAG:-r6}/sol_cfg4 ARGS="--agents 4096 --envs 16" bash scripts/gpu_sol.sh > $O/sol_cfg4.log 2>&1 || { echo "STOP sol_cfg4"; tail -5 $O/sol_cfg4.log; exit 1; }; head -30 $O/sol_cfg4/sol.md ;;
    sol_cfg5) TAG=${TAG:-r6}/sol_cfg5 ARGS="--agents 1024 --envs 64 --dim 3 --num_obstacles 8 --dtype fp16" bash scripts/gpu_sol.sh > $O/sol_cfg5.log 2>&1 || { echo "STOP sol_cfg5"; tail -5 $O/sol_cfg5.log; exit 1; }; head -30 $O/sol_cfg5/sol.md ;;
    configs) TAG=${TAG:-r6}/configs bash scripts/gpu_configs.sh || { echo "STOP configs"; exit 1; } ;;
    dp:*)
      NR=${s#dp:} STEPS=3 bash scripts/gpu_dp_rehearsal.sh || { echo "STOP $s"; exit 1; }
      mv gpurun_out/dp${s#dp:}_rehearsal.log $O/ ;;
    neg)
      MACBF_EXT=alt_so/shrink/_C.so timeout -k 10 600 python -u -m pytest tests/test_gpu_scan_plans.py -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/neg.log 2>&1
      rc=$?; tail -3 $O/neg.log
      if [ $rc -eq 1 ]; then echo "neg: the shrunk search box FAILS the oracle tests (expected)"; else echo "STOP neg rc=$rc (expected 1)"; exit 1; fi ;;
    py:*)
      spec=${s#py:}; scr=${spec%%,*}; args=""; [ "$spec" != "$scr" ] && args=${spec#*,}
      L=$O/py_${scr%.py}_$(echo "$args" | tr -c 'a-zA-Z0-9' _).log
      timeout -k 10 300 python -u scripts/$scr ${args//,/ } > $L 2>&1 || { echo "STOP $s"; tail -5 $L; exit 1; }
      echo "== $s"; tail -25 $L ;;
    sl:*)
      kv=${s#sl:}; n=sl_$(echo "$kv" | tr -c 'a-zA-Z0-9' _)
      env "$kv" timeout -k 10 300 $B --envs 8 > $O/$n.log 2>&1 || { echo "STOP $n"; tail -5 $O/$n.log; exit 1; }
      echo "$n: $(ms $O/$n.log)" ;;
    e:*)
      spec=${s#e:}; kv=${spec%%:*}; sub=${spec#*:}
      PFX="$(echo "$kv" | tr -c 'a-zA-Z0-9' _)_" STEPS="$sub" TAG=${TAG:-r6} env "$kv" bash scripts/gpu_steps.sh | grep -v '^DONE' || exit 1 ;;
    env:*) export "${s#env:}" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo DONE
