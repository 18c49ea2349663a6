#!/bin/bash
# Safety study: train from random init, then evaluate with and without
# test-time refinement; per-term controller gradient norms on the oracle. -> gpurun_out/eval/
set -e -o pipefail
O=gpurun_out/eval
mkdir -p $O
S="python -u scripts/safety_study.py"
timeout -k 10 300 $S train --name headline --agents 1024 --envs 64 --steps ${HEAD_STEPS:-4000} --out $O > $O/train_headline.log 2>&1
timeout -k 10 180 $S train --name alt10 --agents 1024 --envs 64 --steps ${VAR_STEPS:-2000} --alternate_every 10 --out $O > $O/train_alt10.log 2>&1
timeout -k 10 180 $S train --name nobptt --agents 1024 --envs 64 --steps ${VAR_STEPS:-2000} --no_bptt --out $O > $O/train_nobptt.log 2>&1
timeout -k 10 150 $S train --name cfg2 --agents 32 --envs 1 --steps 6000 --display 500 --out $O > $O/train_cfg2.log 2>&1
timeout -k 10 400 $S eval --models none,$O/headline.pt,$O/alt10.pt,$O/nobptt.pt,$O/cfg2.pt --agents 1024 --episodes ${EPISODES:-10} --out $O --tag eval1024 > $O/eval1024.log 2>&1
timeout -k 10 200 $S grads --models none,$O/headline.pt --agents 1024 --envs 4 --iters 2 --out $O --tag grads > $O/grads.log 2>&1
