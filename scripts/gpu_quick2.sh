# quick perf check: micro (fp32) + bench fp32 with phases + kernel stats
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-q2}
mkdir -p $O
timeout -k 10 300 python scripts/micro_step.py --dtype ${DT:-fp32} --tag $TAG > $O/micro.log 2>&1 || { tail -5 $O/micro.log; exit 1; }
tail -1 $O/micro.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype ${DT:-fp32} --phases > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.log').read().strip().split(chr(10))[-1]); print(round(d['ms_per_step'],3), round(d['value']/1e6,2), d.get('phases_ms'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --dtype ${DT:-fp32} > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
python3 - <<'PY'
import csv, os
p = os.environ['GRAFT_REPO_ROOT'] + '/' + os.environ.get('O_REL', 'gpurun_out/' + os.environ.get('TAG', 'q2')) + '/prof/run_kernel_stats.csv'
for r in list(csv.DictReader(open(p)))[:12]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f} us {float(r['Percentage']):6.2f}%")
PY
