#!/bin/bash
# Round 5 batch 10: phase clocks of the x3 controller step (scripts/stamps_ctrl.py), forward tests
# after the stamps plumbing. Output: gpurun_out/${TAG:-r5b10}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b10}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_runtime.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; if [ $rc -ne 0 ]; then echo "STOP tests"; exit $rc; fi
timeout -k 10 200 python scripts/stamps_ctrl.py > $O/stamps_ctrl.log 2>&1 && tail -10 $O/stamps_ctrl.log || { echo STOP stamps; tail -5 $O/stamps_ctrl.log; exit 1; }
timeout -k 10 200 python scripts/stamps_ctrl.py --step 2 > $O/stamps_ctrl_s2.log 2>&1 && tail -10 $O/stamps_ctrl_s2.log || { echo STOP stamps; exit 1; }
