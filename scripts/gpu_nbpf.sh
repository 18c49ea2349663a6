# Node backward next-chunk pooled-row prefetch (build/variants/nbpf, -DNB_PREFETCH=1) vs in-tree:
# fp32 GPU tests with the variant, then interleaved per-step micro-benchmark. Output: gpurun_out/nbpf
cd $GRAFT_REPO_ROOT
O=gpurun_out/nbpf
mkdir -p $O
MACBF_EXT=$GRAFT_REPO_ROOT/build/variants/nbpf/_C.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fp32.py tests/test_gpu_runtime.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  timeout -k 10 300 python scripts/micro_step.py --tag base_$rep >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
  MACBF_EXT=$GRAFT_REPO_ROOT/build/variants/nbpf/_C.so timeout -k 10 300 python scripts/micro_step.py --so build/variants/nbpf/_C.so --tag nbpf_$rep >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
done
grep '^{' $O/micro.log | python -c "import sys,json; [print(d['tag'], d['node_bwd'], d['edge_bwd']) for d in map(json.loads, sys.stdin)]"
