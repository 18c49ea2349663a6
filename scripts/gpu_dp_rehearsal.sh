# Multi-rank rehearsal of the benchmark on ONE GPU: NR ranks (default 8) share the device over
# gloo (RCCL places one rank per GPU; the driver runs the real 1/2/4/8-GPU RCCL scaling at round
# end). Default: BASELINE config #3 as stated, 64 envs split over the ranks (--global_envs 64,
# strong scaling). Exercises the torchrun launch, per-rank sampling, async count all-reduce,
# gradient all-reduce, max-over-ranks timing and the rank-0 JSON line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NR=${NR:-8}
MACBF_DP_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NR \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $NR --steps ${STEPS:-5} --warmup 2 \
  --global_envs ${GENVS:-64} > gpurun_out/dp${NR}_rehearsal.log 2>&1
rc=$?
tail -2 gpurun_out/dp${NR}_rehearsal.log
exit $rc
