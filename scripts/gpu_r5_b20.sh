#!/bin/bash
# Round 5 batch 20 (diagnostics): controller-step phase clocks without the pooled-row / argmax
# stores (alt_so/nopst, -DCTRL_DIAG_NOPOOLSTORE=1: wrong results, clocks only) against the
# in-tree build. Output: gpurun_out/${TAG:-r5b20}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b20}
mkdir -p $O
timeout -k 10 200 python scripts/stamps_ctrl.py > $O/stamps_cur.log 2>&1 && tail -9 $O/stamps_cur.log | head -8 || { echo STOP stamps; exit 1; }
MACBF_SELFCHECK=0 MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/nopst/_C.so timeout -k 10 200 python scripts/stamps_ctrl.py > $O/stamps_nopst.log 2>&1 && tail -9 $O/stamps_nopst.log | head -8 || { echo STOP stamps; tail -3 $O/stamps_nopst.log; exit 1; }
