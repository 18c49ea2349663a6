#!/bin/bash
# GPU suite, then every BASELINE config with this binary (scripts/gpu_configs.sh).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r4f}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -6 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
TAG=${TAG:-r4f}/configs bash scripts/gpu_configs.sh
