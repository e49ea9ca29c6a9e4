#!/bin/bash
# Round 4: A/B of the phase-4 layout variant, then the round-4 profile of the main library.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS="main p4" REPS="1 2" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r4g_ab.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4_profile.sh 2>&1 | tee gpurun_out/r4g_profile.log
exit ${PIPESTATUS[0]}
