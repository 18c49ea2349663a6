#!/bin/bash
# Round 5 batch 23 (diagnostics): 3-D scan culling counts split by reason (kNN vs safety only).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b23}
mkdir -p $O
timeout -k 10 200 python scripts/stamps_scan.py --dim 3 --obstacles 8 > $O/stamps_scan_3d.log 2>&1 && tail -14 $O/stamps_scan_3d.log || { echo STOP; tail -3 $O/stamps_scan_3d.log; exit 1; }
timeout -k 10 200 python scripts/stamps_scan.py > $O/stamps_scan_2d.log 2>&1 && tail -14 $O/stamps_scan_2d.log
