# Strong-scaling per-rank slices of BASELINE config #3 (64 envs over DP 2/4/8 -> 32/16/8 envs per
# GPU) with the final kernels, fp32 and bf16. Output: gpurun_out/slices_final
cd $GRAFT_REPO_ROOT
O=gpurun_out/slices_final
mkdir -p $O
for dt in fp32 bf16; do
  for e in 32 16 8; do
    timeout -k 10 300 python bench.py --envs $e --steps 20 --warmup 5 --dtype $dt > $O/slice_${dt}_$e.log 2>&1 || { tail -5 $O/slice_${dt}_$e.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/slice_${dt}_$e.log').read().strip().split(chr(10))[-1]); print('$dt envs $e', round(d['ms_per_step'],3), round(d['value']/1e6,1), 'T', d['mean_T'])"
  done
done
