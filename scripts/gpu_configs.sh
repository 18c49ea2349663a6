#!/bin/bash
# Every BASELINE.json config with ONE binary in ONE GPU call, one JSON line
# each (bench.py's own), 20 timed steps after 5 warm-up steps unless stated:
#   #1  8 agents, CPU reference path (oracle engine), 1 training iteration (train.py, plumbing)
#   #2  32 agents x 1 env, bf16 (the BASELINE precision) and fp32
#   #3  1024 agents x 64 envs: fp32 (headline) and bf16; the 8-env slice config #3 has per GPU at DP 8
#   #4  4096 agents x 16 envs (LDS neighbour-tile stress), fp32
#   #5  1024 agents x 64 envs, 3-D + 8 obstacles x 12 points, fp16 (dynamic loss scaling) and fp32
# Output: gpurun_out/${TAG:-configs}/cfg*.log and configs.jsonl
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-configs}
mkdir -p $O
: > $O/configs.jsonl
run() {   # name, timeout, bench args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -5 $O/$name.log; exit 1; }
  local line=$(grep '^{' $O/$name.log | tail -1)
  python - "$name" "$line" >> $O/configs.jsonl <<'PY'
import json, sys
d = json.loads(sys.argv[2]); d["cfg"] = sys.argv[1]; print(json.dumps(d))
PY
  python -c "import json,sys; d=json.loads(sys.argv[1]); print(f\"{sys.argv[2]:14s} {d['ms_per_step']:8.3f} ms  {d['value']/1e6:8.2f} M agent-steps/s  safety {d['safety_rate']:.4f}  T {d['mean_T']:.1f}  {d['dtype']}\")" "$line" "$name"
}
# #1: CPU oracle engine, 8 agents, one iteration (train.py, the reference CLI) + the bench on CPU
timeout -k 10 300 python train.py --num_agents 8 --device cpu --train_steps 1 --display_steps 1 > $O/cfg1_train.log 2>&1 || { echo "FAILED cfg1"; tail -5 $O/cfg1_train.log; exit 1; }
echo "cfg1_train     ok: $(grep -c loss $O/cfg1_train.log) log line(s)"
run cfg1_cpu 300 --device cpu --agents 8 --envs 1 --steps 3 --warmup 1
run cfg2_bf16 300 --agents 32 --envs 1 --steps 30 --warmup 5 --dtype bf16
run cfg2_fp32 300 --agents 32 --envs 1 --steps 30 --warmup 5
run cfg3_fp32 300 --agents 1024                  # bench.py's default: 64 envs over the ranks (here one)
run cfg3_bf16 300 --agents 1024 --dtype bf16
run cfg3_slice8_fp32 300 --agents 1024 --envs 8
run cfg4_fp32 300 --agents 4096 --envs 16
run cfg5_fp16 300 --agents 1024 --envs 64 --dim 3 --num_obstacles 8 --dtype fp16
run cfg5_fp32 300 --agents 1024 --envs 64 --dim 3 --num_obstacles 8
run cfg3_fixedT_fp32 300 --agents 1024 --no_early_stop
run cfg3_fixedT_bf16 300 --agents 1024 --no_early_stop --dtype bf16
