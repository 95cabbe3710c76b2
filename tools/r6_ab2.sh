#!/bin/bash
# round-5 HEAD vs current vs workgroup barriers every 1 / 2 ring blocks in the GEMV stream (TI_GEMV_SYNC)
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/turboinfer_amd
bash tools/r6_ab.sh r6ab2 r5=$L/lib_r5/libturboinfer_amd.so cur=. sync1=$L/lib_sync1/libturboinfer_amd.so sync2=$L/lib_sync2/libturboinfer_amd.so
