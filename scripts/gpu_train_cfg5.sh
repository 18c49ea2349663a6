# Training-quality runs of BASELINE config #5 (1024 agents x 64 envs, 3-D double integrator, 8
# static obstacles x 12 points) with the reference CLI: fp16 mixed precision (the config's
# precision, dynamic loss scaling) and fp32 (x3), JSONL logs every 100 steps. Output: gpurun_out/cfg5
cd $GRAFT_REPO_ROOT
O=gpurun_out/cfg5
mkdir -p $O
timeout -k 10 500 python -u train.py --num_agents 1024 --num_envs 64 --dim 3 --num_obstacles 8 --dtype fp16 \
  --train_steps ${STEPS:-3000} --display_steps 100 --log_path $O/cfg5_3d_obs_fp16.jsonl > $O/fp16.log 2>&1 || { tail -5 $O/fp16.log; exit 1; }
tail -c 700 $O/cfg5_3d_obs_fp16.jsonl
timeout -k 10 500 python -u train.py --num_agents 1024 --num_envs 64 --dim 3 --num_obstacles 8 --dtype fp32 \
  --train_steps ${STEPS:-3000} --display_steps 100 --log_path $O/cfg5_3d_obs_fp32.jsonl > $O/fp32.log 2>&1 || { tail -5 $O/fp32.log; exit 1; }
tail -c 700 $O/cfg5_3d_obs_fp32.jsonl
