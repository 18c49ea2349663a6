# Multi-rank rehearsal of the benchmark on ONE GPU: 2 ranks share the device over gloo (RCCL
# places one rank per GPU; the driver runs the real 1/2/4/8-GPU RCCL scaling at round end).
# Exercises the torchrun launch, per-rank sampling, async count all-reduce, gradient
# all-reduce, max-over-ranks timing and the rank-0 JSON line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MACBF_DP_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --envs 16 \
  > gpurun_out/dp_rehearsal.log 2>&1
rc=$?
tail -2 gpurun_out/dp_rehearsal.log
exit $rc
