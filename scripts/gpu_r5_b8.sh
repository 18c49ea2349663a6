#!/bin/bash
# Round 5 batch 8 (VERDICT r4 item 3 evidence): the kNN scan at the occupancy a fused scan +
# controller-step kernel would give it (alt_so/fuseprobe, -DSCAN_FUSE_PROBE=1): scan tests with the
# variant (same lists), then kernel traces of the headline with both builds.
# Output: gpurun_out/${TAG:-r5b8}/
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r5b8}
mkdir -p $O
MACBF_EXT=alt_so/fuseprobe/_C.so timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -q -p no:cacheprovider -k scan --timeout 200 --timeout-method thread > $O/probe_tests.log 2>&1
rc=$?; tail -2 $O/probe_tests.log; if [ $rc -ne 0 ]; then echo "STOP probe tests"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
for v in cur probe; do
  if [ $v = probe ]; then export MACBF_EXT=$GRAFT_REPO_ROOT/alt_so/fuseprobe/_C.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  cp $(find $O/prof_$v -name "*kernel_stats.csv" | head -1) $O/kernel_stats_$v.csv
  python3 $GRAFT_REPO_ROOT/scripts/kstats.py $O/kernel_stats_$v.csv 8 | grep -i "scan\|ctrl_fwd"
done
# early-stop wait without the per-wait hipStreamQuery (MACBF_POLL_QUERY_MS=100): kernel trace
# (gap after each controller step) and interleaved headline A/B
unset MACBF_EXT
MACBF_POLL_QUERY_MS=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_poll -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $O/prof_poll.log 2>&1 || { tail -5 $O/prof_poll.log; exit 1; }
cp $(find $O/prof_poll -name "*kernel_trace.csv" | head -1) $O/kernel_trace_poll.csv
cp $(find $O/prof_cur -name "*kernel_trace.csv" | head -1) $O/kernel_trace_cur.csv
cd $GRAFT_REPO_ROOT
ms() { grep '^{' $1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))'; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/poll0_$rep.log 2>&1 || { echo STOP; exit 1; }
  MACBF_POLL_QUERY_MS=100 timeout -k 10 200 python bench.py > $O/poll100_$rep.log 2>&1 || { echo STOP; exit 1; }
  echo "poll $rep q0 $(ms $O/poll0_$rep.log) q100 $(ms $O/poll100_$rep.log)"
done
