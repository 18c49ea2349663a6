#!/bin/bash
# Round 5 batch 18: a kernel's back-to-back weight copies (LDS-DMA) wait once after the last one
# (alt_so/onewait, -DMB_COPY_ONEWAIT=1): the whole GPU suite with the variant, controller-step and
# node-backward phase clocks, interleaved headline fp32 x3 / bf16 x2. Output: gpurun_out/${TAG:-r5b18}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5b18}
mkdir -p $O
ALT=${ALT:-onewait}
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$ALT/_C.so timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests_alt.log 2>&1
rc=$?; tail -1 $O/tests_alt.log; if [ $rc -ne 0 ]; then echo "STOP alt tests"; exit $rc; fi
MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$ALT/_C.so timeout -k 10 200 python scripts/stamps_ctrl.py > $O/stamps_ctrl_alt.log 2>&1 && tail -9 $O/stamps_ctrl_alt.log | head -2 || { echo STOP stamps; exit 1; }
MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$ALT/_C.so timeout -k 10 200 python scripts/stamps_node.py --node16 --envs 64 > $O/stamps_node_alt.log 2>&1 && grep -m1 weights $O/stamps_node_alt.log || { echo STOP stamps; exit 1; }
for rep in 1 2 3; do
  for dt in fp32 bf16; do
    if [ $dt = bf16 ] && [ $rep = 3 ]; then continue; fi
    timeout -k 10 200 python bench.py --dtype $dt > $O/cur_${dt}_$rep.log 2>&1 || { echo STOP; exit 1; }
    MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/$ALT/_C.so timeout -k 10 200 python bench.py --dtype $dt > $O/alt_${dt}_$rep.log 2>&1 || { echo STOP; exit 1; }
    echo "$dt $rep cur $(ms $O/cur_${dt}_$rep.log) alt $(ms $O/alt_${dt}_$rep.log)"
  done
done
