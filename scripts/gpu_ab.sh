# Interleaved A/B benchmark of engine scheduling knobs in one GPU call (same box, same clocks).
# usage: bash scripts/gpu_ab.sh TAG ROUNDS "ENV_A" "ENV_B" ["ENV_C" ...]
#   e.g. bash scripts/gpu_ab.sh ab1 3 "MACBF_REDUCE_LATE=0" "MACBF_REDUCE_LATE=4"
TAG=$1; ROUNDS=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.log
: > $OUT
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    line=$(env $v timeout -k 10 120 python bench.py --steps 20 --warmup 3 2>/dev/null | tail -1) || { echo "FAIL $v" >> $OUT; exit 1; }
    ms=$(echo "$line" | python -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"], 3))')
    echo "$r | $v | $ms" | tee -a $OUT
  done
done
