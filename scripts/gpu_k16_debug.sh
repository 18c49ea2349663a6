#!/bin/bash
# 1-pass 16x16x32 kernels after the wave_id() fix: the MFMA/EXEC probe, diagnostics
# (scripts/diag_k16_1pass.py), the GPU suite, the no-sched-barrier builds on the oracle tests,
# then the headline benches (bf16 default and two-workgroups-per-CU variant, fp32, cfg5 fp16).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-k16dbg}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc ($2)"; exit $rc; fi; }
timeout -k 10 120 python -u -m pytest tests/test_gpu_probe.py -q -s -p no:cacheprovider --timeout 60 --timeout-method thread -k mfma_under > $O/probe.log 2>&1; ok $? probe
grep -E "VGPR|passed|failed" $O/probe.log
for dt in bf16 fp16; do
  timeout -k 10 120 python -u scripts/diag_k16_1pass.py --dtype $dt > $O/diag_$dt.json 2> $O/diag_$dt.err; ok $? diag_$dt
done
python - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/diag_*.json")):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(os.path.basename(f), "unreadable", e); continue
    keys = [k for k in d if k.endswith("_rel") or "nan" in k or k in ("edge_k16_vs_k32_grad",)]
    print(os.path.basename(f), {k: (round(d[k], 4) if isinstance(d[k], float) else d[k]) for k in keys})
PY
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -15 $O/gpu_tests.log; ok $rc tests
b() { local name=$1; shift; env "$@" > $O/$name.log 2>&1; local rc=$?; ok $rc $name; grep '^{' $O/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['ms_per_step'],3), 'ms', d['dtype'])"; }
b bench_bf16 timeout -k 10 300 python bench.py --dtype bf16
b bench_bf16_wg2 MACBF_EXT=alt_so/k16wg2/_C.so timeout -k 10 300 python bench.py --dtype bf16
b bench_fp32 timeout -k 10 300 python bench.py
b bench_cfg5_fp16 timeout -k 10 300 python bench.py --dim 3 --num_obstacles 8 --dtype fp16
b bench_bf16_b timeout -k 10 300 python bench.py --dtype bf16
