# BASELINE configs on one MI355X: #2 (32 agents), #3 per-GPU slice (1024 x 64), #4 (4096 agents),
# #5 (3-D + 8 obstacles, bf16 and fp16).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --agents 32 --envs 1 --steps 20 --warmup 3 > gpurun_out/cfg2_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --agents 32 --envs 64 --steps 20 --warmup 3 > gpurun_out/cfg2b_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --agents 4096 --envs 16 --steps 10 --warmup 3 --phases > gpurun_out/cfg4_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --agents 1024 --envs 64 --steps 10 --warmup 3 --no_early_stop --phases > gpurun_out/cfg3_fixedT_bench.log 2>&1 || exit $?
tail -n1 gpurun_out/cfg2_bench.log gpurun_out/cfg2b_bench.log gpurun_out/cfg4_bench.log gpurun_out/cfg3_fixedT_bench.log
timeout -k 10 300 python bench.py --agents 1024 --envs 64 --dim 3 --num_obstacles 8 --steps 10 --warmup 3 --phases > gpurun_out/cfg5_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --agents 1024 --envs 64 --dim 3 --num_obstacles 8 --dtype fp16 --steps 10 --warmup 3 --phases > gpurun_out/cfg5_fp16_bench.log 2>&1 || exit $?
tail -n1 gpurun_out/cfg5_bench.log gpurun_out/cfg5_fp16_bench.log
