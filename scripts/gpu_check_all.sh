#!/bin/bash
# Full GPU check: the GPU test suite, the headline bench (20 timed steps after 5 warm-up steps),
# then a rocprofv3 kernel trace of a short bench. Output: gpurun_out/${TAG:-all}
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-all}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_EXTRA} > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
if [ -z "$NO_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
  python scripts/kstats.py $O/kernel_stats.csv 40
fi
