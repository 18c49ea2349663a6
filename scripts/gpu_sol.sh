#!/bin/bash
# Speed-of-light table of the headline iteration: two PMC passes over
# bench.py ITSELF (--steps 3 --warmup 1, ARGS: extra bench flags), each pass its own rocprofv3 run
# with the program right after --; durations from the same dispatches' timestamps.
# Output: gpurun_out/${TAG:-sol}/sol.md (+ sol.json)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-sol}
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"
cd /tmp && export TMPDIR=/tmp
export MACBF_SELFCHECK=0      # its small start-up dispatches would enter the per-dispatch averages
n=0
for P in "$P1" "$P2"; do
  n=$((n+1))
  timeout -s KILL 240 rocprofv3 --pmc $P -d $O/p$n -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 $ARGS > $O/p$n.log 2>&1 || { tail -5 $O/p$n.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
python scripts/sol_table.py $O/sol.md $(find $O -name "*counter_collection.csv")
