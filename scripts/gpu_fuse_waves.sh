# x3 fused controller step: waves per workgroup (variants f12 / f16) x agents per wave
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-fw}
mkdir -p $O
for rep in 1 2; do
  for cfg in base:32 f12:32 f12:22 f16:16 base:16 f12:16; do
    v=${cfg%%:*}; apw=${cfg#*:}
    if [ $v = base ]; then so=""; else so="--so build/variants/$v/_C.so"; fi
    MACBF_CTRL_APW=$apw timeout -k 10 200 python scripts/micro_step.py --dtype fp32 $so --tag ${v}_apw$apw >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
  done
done
grep '^{' $O/micro.log | python -c "
import sys, json
for d in map(json.loads, sys.stdin):
    print(d['tag'], d.get('ctrl_fwd'), d.get('node_bwd'), d.get('edge_bwd'))"
