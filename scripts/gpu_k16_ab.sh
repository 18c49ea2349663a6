#!/bin/bash
# GPU suite + the 16x16x32 backward kernels in the 1-pass builds, A/B on one box:
#   k16      default build: CBF / edge 16x16x32 at two workgroups per CU (4 waves / SIMD), node 16x16x32
#   k16wg1   alt_so/k16wg1 (scripts/build_variant.sh k16wg1 cbf,ctrl,cbf_f16,ctrl_f16
#            "-DCBF16_WGPC=1 -DE16_WGPC=1"): one workgroup per CU (2 waves / SIMD, no spills)
#   k32      MACBF_CBF16=0 MACBF_EB16=0 MACBF_NODE16=0: the round-3 32x32x16 kernels
# for bf16 at the headline (1024 x 64) and config #2 (32 x 1), fp16 at config #5, fp32 headline.
# Output: gpurun_out/${TAG:-k16ab}/*.log, ab.jsonl. Any step that crashes (not a plain test
# failure) ends the script.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-k16ab}
mkdir -p $O
: > $O/ab.jsonl
step() {   # rc check: 0 ok, 1 test failures (continue), anything else (crash / timeout): stop
  local rc=$1 what=$2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $what rc=$rc"; exit $rc; fi
}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $O/gpu_tests.log 2>&1
  rc=$?; tail -25 $O/gpu_tests.log; step $rc "gpu tests"
fi
bench() {   # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python bench.py "$@" > $O/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED $name rc=$rc"; tail -4 $O/$name.log; step $rc $name; return; fi
  local line=$(grep '^{' $O/$name.log | tail -1)
  python - "$name" "$line" >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads(sys.argv[2]); d["run"] = sys.argv[1]; print(json.dumps(d))
PY
  python -c "import json,sys; d=json.loads(sys.argv[1]); print(f\"{sys.argv[2]:22s} {d['ms_per_step']:8.3f} ms  {d['value']/1e6:8.2f} M/s  {d['dtype']}\")" "$line" "$name"
}
K32="MACBF_CBF16=0 MACBF_EB16=0 MACBF_NODE16=0"
WG1="MACBF_EXT=alt_so/k16wg1/_C.so MACBF_EDGE_WG_PER_CU=1"
for rep in 1 2; do
  bench bf16_k16_$rep "X=1" --dtype bf16
  bench bf16_k16wg1_$rep "$WG1" --dtype bf16
  bench bf16_k32_$rep "$K32" --dtype bf16
done
bench cfg2_bf16_k16 "X=1" --agents 32 --envs 1 --steps 30 --warmup 5 --dtype bf16
bench cfg2_bf16_k32 "$K32" --agents 32 --envs 1 --steps 30 --warmup 5 --dtype bf16
bench cfg5_fp16_k16 "X=1" --agents 1024 --envs 64 --dim 3 --num_obstacles 8 --dtype fp16
bench cfg5_fp16_k32 "$K32" --agents 1024 --envs 64 --dim 3 --num_obstacles 8 --dtype fp16
bench fp32_k16 "X=1"
exit 0
