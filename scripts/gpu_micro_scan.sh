cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_forward.py -q -m gpu -p no:cacheprovider -k scan > gpurun_out/ms_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ms_tests.log; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/micro_scan.py 1024 && timeout -k 10 300 python scripts/micro_scan.py 4096 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES -d $GRAFT_REPO_ROOT/gpurun_out/pmc_scan -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/micro_scan.py 1024 > $GRAFT_REPO_ROOT/gpurun_out/ms_pmc.log 2>&1
echo "pmc rc=$?"
