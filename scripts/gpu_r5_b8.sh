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
