#!/bin/bash
# Round 5 batch 34: alt_so/g24b = 2-D 24^2 cell grid in blocks of >= 576 threads (16^2 below) vs
# in-tree (16^2). Full GPU suite on the variant, interleaved headline fp32 x2, slice x1, bf16 x1.
# Output: gpurun_out/${TAG:-r5b34}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b34}
mkdir -p $O
X=$GRAFT_REPO_ROOT/alt_so/g24b/_C.so
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
MACBF_EXT=$X timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/gpu_tests_g24b.log 2>&1
rc=$?; tail -n 2 $O/gpu_tests_g24b.log; if [ $rc -ne 0 ]; then echo "STOP tests"; exit $rc; fi
for rep in 1 2; do
  timeout -k 10 200 python bench.py > $O/cur_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_EXT=$X timeout -k 10 200 python bench.py > $O/g24b_fp32_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "fp32 $rep cur $(ms $O/cur_fp32_$rep.log) g24b $(ms $O/g24b_fp32_$rep.log)"
done
timeout -k 10 200 python bench.py --dtype bf16 > $O/cur_bf16.log 2>&1 || { echo STOP; exit 1; }
MACBF_EXT=$X timeout -k 10 200 python bench.py --dtype bf16 > $O/g24b_bf16.log 2>&1 || { echo STOP; exit 1; }
echo "bf16 cur $(ms $O/cur_bf16.log) g24b $(ms $O/g24b_bf16.log)"
timeout -k 10 200 python bench.py --agents 1024 --envs 8 > $O/cur_slice.log 2>&1 || { echo STOP; exit 1; }
MACBF_EXT=$X timeout -k 10 200 python bench.py --agents 1024 --envs 8 > $O/g24b_slice.log 2>&1 || { echo STOP; exit 1; }
echo "slice cur $(ms $O/cur_slice.log) g24b $(ms $O/g24b_slice.log)"
