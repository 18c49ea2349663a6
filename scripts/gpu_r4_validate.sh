#!/bin/bash
# Round-4 validation after the MFMA hazard fixes (wave_id, compile-time stamps, routed edge db2):
# GPU suite; the no-sched-barrier builds on the float64-oracle tests; A/B of the 16x16x32 vs the
# 32x32x16 backward kernels in bf16 / fp16 (interleaved, same box); fp32 headline; phase clocks.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r4v}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc ($2)"; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -8 $O/gpu_tests.log; ok $rc tests
: > $O/ab.jsonl
b() { local name=$1; shift; env "$@" > $O/$name.log 2>&1; local rc=$?; ok $rc $name
  local line=$(grep '^{' $O/$name.log | tail -1)
  python - "$name" "$line" >> $O/ab.jsonl <<'PY'
import json, sys
d = json.loads(sys.argv[2]); d["run"] = sys.argv[1]; print(json.dumps(d))
PY
  python -c "import json,sys; d=json.loads(sys.argv[1]); print(f\"{sys.argv[2]:18s} {d['ms_per_step']:7.3f} ms  T {d['mean_T']:.2f}  {d['dtype']}\")" "$line" "$name"; }
K32="MACBF_CBF16=0 MACBF_EB16=0 MACBF_NODE16=0"
for rep in 1 2; do
  b bf16_k16_$rep X=1 timeout -k 10 300 python bench.py --dtype bf16
  b bf16_k32_$rep $K32 timeout -k 10 300 python bench.py --dtype bf16
done
b cfg5_fp16_k16 X=1 timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16
b cfg5_fp16_k32 $K32 timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16
b cfg2_bf16_k16 X=1 timeout -k 10 300 python bench.py --agents 32 --envs 1 --steps 30 --warmup 5 --dtype bf16
b cfg2_bf16_k32 $K32 timeout -k 10 300 python bench.py --agents 32 --envs 1 --steps 30 --warmup 5 --dtype bf16
b fp32_1 X=1 timeout -k 10 300 python bench.py
b fp32_2 X=1 timeout -k 10 300 python bench.py
timeout -k 10 200 python -u scripts/stamps_node.py --node16 --envs 64 > $O/stamps16.log 2>&1; ok $? stamps16
tail -18 $O/stamps16.log
timeout -k 10 200 python -u scripts/stamps_cbf.py > $O/stamps_cbf.log 2>&1; ok $? stamps_cbf
tail -12 $O/stamps_cbf.log
