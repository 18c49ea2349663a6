# fp16 mixed-precision cycle: GPU tests, then the headline config in bf16 and fp16 and
# BASELINE config #5 (3-D + 8 obstacles) in fp16.  usage: bash scripts/gpu_fp16.sh TAG [tests...]
TAG=${1:-fp16}; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TESTS=${@:-tests/test_gpu_fp16.py}
timeout -k 10 900 python -m pytest $TESTS -q -m gpu -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log
tail -8 gpurun_out/${TAG}_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for cfg in "bf16:" "fp16:" "fp16:--dim 3 --num_obstacles 8"; do
  dt=${cfg%%:*}; extra=${cfg#*:}
  name=${TAG}_bench_${dt}$(echo $extra | tr -d ' -')
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 --phases --dtype $dt $extra > gpurun_out/${name}.log 2>&1
  rc=$?
  echo "bench rc=$rc" >> gpurun_out/${name}.log
  tail -2 gpurun_out/${name}.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
