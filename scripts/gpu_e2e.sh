# End-to-end CLI checks on the GPU box: smoke(), torchrun bench, train + resume, evaluate.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2e
O=gpurun_out/e2e
timeout -k 10 600 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 > $O/torchrun.log 2>&1 || { tail -20 $O/torchrun.log; exit 1; }
tail -1 $O/torchrun.log | cut -c1-160
timeout -k 10 300 python train.py --num_agents 64 --num_envs 8 --train_steps 30 --model_path $O/ck.pt --log_path $O/log.jsonl --display_steps 10 --save_steps 15 > $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
timeout -k 10 300 python train.py --num_agents 64 --num_envs 8 --train_steps 40 --model_path $O/ck.pt --log_path $O/log2.jsonl --display_steps 10 --save_steps 100 > $O/train2.log 2>&1 || { tail -20 $O/train2.log; exit 1; }
tail -2 $O/log.jsonl | cut -c1-300; tail -1 $O/log2.jsonl | cut -c1-300
timeout -k 10 300 python evaluate.py --num_agents 64 --model_path $O/ck.pt --episodes 2 > $O/eval.log 2>&1 || { tail -20 $O/eval.log; exit 1; }
tail -3 $O/eval.log
