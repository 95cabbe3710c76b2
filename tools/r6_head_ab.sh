#!/bin/bash
# Round 6: HEAD against the library of an earlier commit (turboinfer_amd/lib_prev, built from a git worktree),
# interleaved on one box
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/r6_ab.sh ${1:-r6head} head=. prev=turboinfer_amd/lib_prev/libturboinfer_amd.so
