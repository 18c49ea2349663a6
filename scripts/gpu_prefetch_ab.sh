cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pf
timeout -k 10 300 python -u -m pytest tests/test_gpu_nd.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pf/nd.log 2>&1 || { echo STOP nd; tail -5 gpurun_out/pf/nd.log; exit 1; }
tail -2 gpurun_out/pf/nd.log
for rep in 1 2; do for m in 1 0 2; do
  MACBF_PREFETCH=$m timeout -k 10 300 python bench.py > gpurun_out/pf/h${m}_${rep}.log 2>&1 || { echo STOP $m; tail -3 gpurun_out/pf/h${m}_${rep}.log; exit 1; }
  echo "head m=$m rep=$rep $(grep '^{' gpurun_out/pf/h${m}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done; done
for m in 1 0 2; do
  MACBF_PREFETCH=$m timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > gpurun_out/pf/c5_${m}.log 2>&1 || { echo STOP c5 $m; tail -3 gpurun_out/pf/c5_${m}.log; exit 1; }
  echo "cfg5 m=$m $(grep '^{' gpurun_out/pf/c5_${m}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
