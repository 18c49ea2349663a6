# A/B of the controller edge-phase agents-per-wave at the headline (fp32): micro + bench per value
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-apw}
mkdir -p $O
for rep in 1 2; do
for apw in ${APWS:-32 16 8}; do
  MACBF_CTRL_APW=$apw timeout -k 10 200 python scripts/micro_step.py --dtype ${DT:-fp32} --tag apw$apw >> $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
done
done
grep '^{' $O/micro.log | python -c "import sys,json; [print(d['tag'], d['ctrl_fwd']) for d in map(json.loads, sys.stdin)]"
for apw in ${APWS:-32 16 8}; do
  MACBF_CTRL_APW=$apw timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype ${DT:-fp32} > $O/bench_$apw.log 2>&1 || { tail -5 $O/bench_$apw.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$apw.log').read().strip().split(chr(10))[-1]); print('apw $apw', round(d['ms_per_step'],3), round(d['value']/1e6,2))"
done
