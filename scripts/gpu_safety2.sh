#!/bin/bash
# Safety study, part 2: a longer headline run, then every checkpoint evaluated with no refinement,
# action refinement and gain-only refinement (1024 agents, 10 episodes). -> gpurun_out/eval2/
set -e -o pipefail
O=gpurun_out/eval2
mkdir -p $O
S="python -u scripts/safety_study.py"
timeout -k 10 540 $S train --name headline_16k --agents 1024 --envs 64 --steps ${HEAD_STEPS:-16000} --display 500 --out $O > $O/train_headline_16k.log 2>&1
M=none,checkpoints/headline_4k.pt,$O/headline_16k.pt,checkpoints/alt10_2k.pt,checkpoints/nobptt_2k.pt,checkpoints/cfg2_6k.pt
timeout -k 10 500 $S eval --models $M --agents 1024 --episodes ${EPISODES:-10} --out $O --tag eval1024 > $O/eval1024.log 2>&1
