#!/bin/bash
# Round-5 baseline on a fresh box: GPU suite, then the sampler-prefetch A/B at the headline
# (MACBF_PREFETCH 0 inline / 1 side stream at once / 2 side stream after the enqueued work),
# interleaved, then a kernel trace of the default headline bench (20 timed steps).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5base}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -4 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
for r in 1 2; do
  for m in 0 1 2; do
    MACBF_PREFETCH=$m timeout -k 10 200 python bench.py > $O/pf${m}_$r.log 2>&1 || { echo "FAILED pf$m"; tail -5 $O/pf${m}_$r.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['ms_per_step'],3))" $O/pf${m}_$r.log "prefetch=$m round $r"
  done
done
TAG=${TAG:-r5base}/prof STEPS=20 bash scripts/gpu_prof.sh > $O/prof_summary.txt 2>&1 && head -30 $O/prof_summary.txt
