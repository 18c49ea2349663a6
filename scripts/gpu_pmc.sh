# PMC counter passes over one short bench run (all kernels). usage: bash scripts/gpu_pmc.sh TAG
TAG=${1:-pmc}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1"; exit $1;; esac; }
rocprofv3 -L > $R/gpurun_out/${TAG}_counters.txt 2>&1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE"
i=1
for P in "$P1" "$P2"; do
  timeout -k 10 400 rocprofv3 --pmc $P -d $R/gpurun_out/${TAG}_p$i -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; fatal $rc
  i=$((i+1))
done
