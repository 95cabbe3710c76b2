#!/bin/bash
# Round 6: the fused launch's K/V ring depth (TI_QA_KV_RING build knob: 3 = HEAD, 2 / 4 = lib_r2 / lib_r4)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/r6_ab.sh r6ring kr3=. kr2=turboinfer_amd/lib_r2/libturboinfer_amd.so kr4=turboinfer_amd/lib_r4/libturboinfer_amd.so
