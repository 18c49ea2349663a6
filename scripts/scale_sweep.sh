#!/usr/bin/env bash
# DP scaling sweep of the headline in ONE allocation (VERDICT r3 missing #3): N = 1/2/4/8 ranks,
# one per GPU over RCCL, weak (--weak: 64 envs per GPU) and strong (BASELINE config #3 as stated,
# bench.py's default: --global_envs 64 sharded over the ranks). One JSON line per run (bench.py's, with world,
# dp_backend, device ids) appended to $OUT. N larger than the visible device count is skipped
# (bench.py would refuse it anyway).
#
#   scripts/scale_sweep.sh [OUT=gpurun_out/scale/scale.jsonl] [STEPS=20] [WARMUP=5] [DTYPE=fp32]
#
# Reference loop that DP shards: /root/reference/train.py:48-105 (one env, one device).
set -uo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/scale/scale.jsonl}
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}
DTYPE=${DTYPE:-fp32}
mkdir -p "$(dirname "$OUT")"
NDEV=$(python -c 'import torch; print(torch.cuda.device_count())')
echo "visible devices: $NDEV" | tee -a "${OUT%.jsonl}.log"
for mode in weak strong; do
  for n in 1 2 4 8; do
    if [ "$n" -gt "$NDEV" ]; then
      echo "skip $mode N=$n (only $NDEV devices)" | tee -a "${OUT%.jsonl}.log"
      continue
    fi
    extra=(--global_envs 64)
    [ "$mode" = weak ] && extra=(--weak)
    echo "== $mode N=$n" | tee -a "${OUT%.jsonl}.log"
    line=$(timeout -k 10 600 python bench.py --gpus "$n" --steps "$STEPS" --warmup "$WARMUP" --dtype "$DTYPE" \
           "${extra[@]}" 2>>"${OUT%.jsonl}.log" | grep '^{')
    rc=$?
    if [ $rc -ne 0 ] || [ -z "$line" ]; then
      echo "FAILED $mode N=$n rc=$rc" | tee -a "${OUT%.jsonl}.log"
      exit 1
    fi
    echo "$line" | tee -a "$OUT"
  done
done
