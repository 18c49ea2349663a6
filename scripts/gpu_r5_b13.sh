#!/bin/bash
# Round 5 batch 13: scan phase clocks and culling counts (scripts/stamps_scan.py), 2-D headline and
# 3-D config #5. Output: gpurun_out/${TAG:-r5b13}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b13}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -q -p no:cacheprovider -k scan --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; if [ $rc -ne 0 ]; then echo "STOP tests"; exit $rc; fi
timeout -k 10 200 python scripts/stamps_scan.py > $O/stamps_scan_2d.log 2>&1 && tail -12 $O/stamps_scan_2d.log || { echo STOP stamps; tail -5 $O/stamps_scan_2d.log; exit 1; }
timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_scan_3d.log 2>&1 && tail -12 $O/stamps_scan_3d.log || { echo STOP stamps; exit 1; }
