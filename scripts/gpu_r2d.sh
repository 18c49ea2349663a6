# Training parity run (HIP fp32 vs oracle) -> forced-RCCL torchrun bench at world 1 -> strong-scaling
# per-rank slices (1024 agents x 32/16/8 envs) -> kernel trace of the 8-env slice.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r2d}
mkdir -p $O
timeout -k 10 900 python -u scripts/parity_run.py --iters 200 --agents 32 --envs 8 --dtype fp32 --out $O/parity_fp32.jsonl > $O/parity_fp32.log 2>&1 || { tail -5 $O/parity_fp32.log; exit 1; }
tail -1 $O/parity_fp32.log | cut -c1-400
MACBF_DP_FORCE_PG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 3 > $O/torchrun_forced_rccl.log 2>&1 || { tail -5 $O/torchrun_forced_rccl.log; exit 1; }
grep metric $O/torchrun_forced_rccl.log | cut -c1-200; grep -o '"dp_backend": "[a-z]*"' $O/torchrun_forced_rccl.log
for d in fp32 bf16; do for e in 32 16 8; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype $d --envs $e --phases > $O/slice_${d}_${e}.log 2>&1 || { tail -5 $O/slice_${d}_${e}.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/slice_${d}_${e}.log').read().strip().split(chr(10))[-1]); print('$d', $e, round(d['ms_per_step'],3), round(d['value']/1e6,2), d.get('phases_ms'))"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --dtype fp32 --envs 8 > $GRAFT_REPO_ROOT/$O/prof8.log 2>&1
echo "prof rc=$?"
