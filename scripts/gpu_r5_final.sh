#!/bin/bash
# Round 5 final measurement: GPU suite, smoke(), every BASELINE config with this
# binary (scripts/gpu_configs.sh) plus the fixed-horizon headline (T = 50, no early stop) in fp32
# and bf16, then a kernel trace of the headline. Output: gpurun_out/${TAG:-r5final}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -4 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || { echo "STOP smoke"; exit 1; }
TAG=${TAG:-r5final}/configs bash scripts/gpu_configs.sh || exit $?
C=$O/configs
for dt in fp32 bf16; do
  timeout -k 10 300 python bench.py --no_early_stop --dtype $dt > $C/cfg3_fixedT_$dt.log 2>&1 || { echo "FAILED fixedT"; exit 1; }
  line=$(grep '^{' $C/cfg3_fixedT_$dt.log | tail -1)
  python - "cfg3_fixedT_$dt" "$line" >> $C/configs.jsonl <<'PY'
import json, sys
d = json.loads(sys.argv[2]); d["cfg"] = sys.argv[1]; print(json.dumps(d))
PY
  python -c "import json,sys; d=json.loads(sys.argv[1]); print(f\"cfg3_fixedT_{sys.argv[2]:5s} {d['ms_per_step']:8.3f} ms  {d['value']/1e6:8.2f} M agent-steps/s\")" "$line" $dt
done
TAG=${TAG:-r5final}/prof STEPS=20 bash scripts/gpu_prof.sh > $O/prof_summary.txt 2>&1 && head -12 $O/prof_summary.txt
