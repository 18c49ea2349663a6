# Round-2 closing verification on one GPU box. Output: gpurun_out/r2_final_b
#   full GPU suite -> smoke() -> headline bench (default flags, fp32) -> bf16 bench ->
#   rocprofv3 kernel stats -> 2-rank gloo rehearsal of the torchrun bench -> 1-rank RCCL torchrun bench
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r2_final_b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-250
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_fp32.log 2>&1 || { tail -5 $O/bench_fp32.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --dtype bf16 > $O/bench_bf16.log 2>&1 || { tail -5 $O/bench_bf16.log; exit 1; }
for f in bench_fp32 bench_bf16; do python -c "import json; d=json.loads(open('$O/$f.log').read().strip().split(chr(10))[-1]); print('$f', round(d['ms_per_step'],3), round(d['value']/1e6,2))"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
MACBF_DP_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --envs 16 > $O/dp_rehearsal.log 2>&1 || { tail -5 $O/dp_rehearsal.log; exit 1; }
tail -1 $O/dp_rehearsal.log | cut -c1-250
MACBF_DP_FORCE_PG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --steps 10 --warmup 3 > $O/rccl1.log 2>&1 || { tail -5 $O/rccl1.log; exit 1; }
tail -1 $O/rccl1.log | cut -c1-250
