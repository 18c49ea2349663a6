#!/bin/bash
# Tie calibration: the tie-aware tests with the allowances off, every measured
# tie / exempt count logged (tests/numerics.py tie_log) -> gpurun_out/${TAG:-r5num}/num.jsonl
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5num}
mkdir -p $O
: > $O/num.jsonl
MACBF_NUM_LOG=$PWD/$O/num.jsonl MACBF_NUM_NOASSERT=1 timeout -k 10 500 python -u -m pytest -q -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_gpu_oracle16.py tests/test_gpu_fp32.py tests/test_gpu_node16.py > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; exit $rc
