#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ab1
mkdir -p $O
PH=$GRAFT_REPO_ROOT/turboinfer_amd/lib_ph/libturboinfer_amd.so
TI_LIB=$PH timeout -k 10 180 python3 tools/stamp_probe.py > $O/ph_7b.txt 2>&1 || { cat $O/ph_7b.txt; exit 1; }
cat $O/ph_7b.txt
TI_LIB=$PH timeout -k 10 180 python3 tools/stamp_probe.py --model tinyllama-1.1b > $O/ph_tl.txt 2>&1 || { cat $O/ph_tl.txt; exit 1; }
cat $O/ph_tl.txt
bash tools/r6_ab.sh r6ab1 r5=$GRAFT_REPO_ROOT/turboinfer_amd/lib_r5/libturboinfer_amd.so cur=.
