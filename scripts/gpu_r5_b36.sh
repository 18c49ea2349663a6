#!/bin/bash
# Round 5 batch 36: the final build (10^3 3-D cells, PC-cell prefix sum): full GPU suite, smoke(),
# headline fp32 / bf16 and config #5 fp16 / fp32 benches. Output: gpurun_out/${TAG:-r5b36}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b36}
mkdir -p $O
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 2 $O/gpu_tests.log; if [ $rc -ne 0 ]; then echo "STOP tests"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log || { echo "STOP smoke"; exit 1; }
timeout -k 10 200 python bench.py > $O/fp32.log 2>&1 || { echo STOP; exit 1; }
timeout -k 10 200 python bench.py --dtype bf16 > $O/bf16.log 2>&1 || { echo STOP; exit 1; }
timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16 > $O/cfg5_fp16.log 2>&1 || { echo STOP; exit 1; }
timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 > $O/cfg5_fp32.log 2>&1 || { echo STOP; exit 1; }
echo "fp32 $(ms $O/fp32.log) bf16 $(ms $O/bf16.log) cfg5 fp16 $(ms $O/cfg5_fp16.log) fp32 $(ms $O/cfg5_fp32.log)"
