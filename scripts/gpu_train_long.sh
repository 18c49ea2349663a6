# Long headline training run with the final round-2 kernels (fp32, reference CLI): 10,000
# iterations with a checkpoint every 5,000, then a resume from that checkpoint to 11,000
# iterations (checkpoint round trip at scale). Output: gpurun_out/train_long
cd $GRAFT_REPO_ROOT
O=gpurun_out/train_long
mkdir -p $O
timeout -k 10 900 python -u train.py --num_agents 1024 --num_envs 64 --train_steps 10000 --display_steps 250 \
  --save_steps 5000 --log_path $O/headline_10k.jsonl --model_path $O/headline.pt > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
tail -c 500 $O/headline_10k.jsonl
timeout -k 10 300 python -u train.py --num_agents 1024 --num_envs 64 --train_steps 11000 --display_steps 250 \
  --save_steps 5000 --log_path $O/headline_resume.jsonl --model_path $O/headline.pt > $O/resume.log 2>&1 || { tail -5 $O/resume.log; exit 1; }
tail -c 500 $O/headline_resume.jsonl
rm -f $O/headline.pt
