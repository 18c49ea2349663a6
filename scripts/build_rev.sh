#!/bin/bash
# The extension as built from the csrc/ of another git revision, for interleaved A/B runs of a
# change against its parent on one GPU box (scripts/gpu_steps.sh ab:NAME, MACBF_EXT=alt_so/NAME/_C.so).
#   scripts/build_rev.sh REV NAME      e.g.  scripts/build_rev.sh HEAD prev
# The Python package of the working tree drives both builds: the revision must be argument-compatible.
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
W=build/rev_$NAME
rm -rf $W && mkdir -p $W/macbf_gnn_amd alt_so/$NAME
git archive "$REV" csrc | tar -x -C $W
python3 $W/csrc/build.py -j 8 > $W/build.log
cp $W/macbf_gnn_amd/_C*.so alt_so/$NAME/_C.so
echo alt_so/$NAME/_C.so
