#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter set, the program right after --) over the fixed
# training workload of scripts/prof_workload.py at ARGS (default: the 8-env DP=8 slice,
# 1024 agents x 8 envs), summarised per kernel. Output: gpurun_out/${TAG:-pmc_cfg}/
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-pmc_cfg}
mkdir -p $O
ARGS=${ARGS:-"--agents 1024 --envs 8"}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"
cd /tmp && export TMPDIR=/tmp
n=0
for P in "$P1" "$P2"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/$O/p$n -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/prof_workload.py --iters 2 $ARGS > $GRAFT_REPO_ROOT/$O/p$n.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/p$n.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
python scripts/prof_workload.py --summarize $(find $O -name "*counter_collection.csv") --out $O/pmc.json > /dev/null
python scripts/pmc_table.py $O/pmc.json > $O/pmc_table.txt; cat $O/pmc_table.txt
