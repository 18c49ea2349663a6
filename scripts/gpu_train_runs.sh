# Training-quality runs with the reference CLI (fp32 default): the headline config and BASELINE
# config #2, JSONL logs (loss terms, accuracies, safety rate, horizon) every display step.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-train}
mkdir -p $O
timeout -k 10 400 python -u train.py --num_agents 1024 --num_envs 64 --train_steps ${STEPS3:-3000} --display_steps 100 \
  --log_path $O/headline_1024x64_fp32.jsonl --model_path $O/headline.pt > $O/headline.log 2>&1 || { tail -5 $O/headline.log; exit 1; }
tail -2 $O/headline.jsonl 2>/dev/null; tail -c 600 $O/headline_1024x64_fp32.jsonl
timeout -k 10 400 python -u train.py --num_agents 32 --num_envs 1 --train_steps ${STEPS2:-10000} --display_steps 250 \
  --log_path $O/cfg2_32x1_fp32.jsonl > $O/cfg2.log 2>&1 || { tail -5 $O/cfg2.log; exit 1; }
tail -c 600 $O/cfg2_32x1_fp32.jsonl
