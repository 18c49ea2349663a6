#!/bin/bash
# Round 5 batch 3: the edge16 register-routed dZ rework (GPU suite + interleaved A/B against
# alt_so/e16old), then a kernel trace of the headline with MACBF_PUBLISH=0 (queue marker + copy
# early stop) to locate the ~6 us gap after every controller step.
cd $GRAFT_REPO_ROOT
TAG=r5e16 ALT=e16old REPS=3 bash scripts/gpu_r5_ab.sh || exit $?
MACBF_PUBLISH=0 TAG=r5e16/pub0 STEPS=6 bash scripts/gpu_prof.sh > gpurun_out/r5e16/pub0_summary.txt 2>&1 && head -8 gpurun_out/r5e16/pub0_summary.txt
