#!/bin/bash
# Round-6 final profiles on HEAD: configs[2] and configs[1] bench + kernel trace (roofline_from_trace, stats) +
# FETCH_SIZE pass (pmc_traffic)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/r6_profile.sh r6fprof_7b || exit 1
bash tools/r6_profile.sh r6fprof_tl --model tinyllama-1.1b || exit 1
