#!/bin/bash
# Round 6: phase stamps of the fused QKV + attention launch (TI_STAMP_PHASES build, TinyLlama)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6qaph
mkdir -p $O
TI_QKV_ATTN=1 TI_LIB=turboinfer_amd/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py --model tinyllama-1.1b > $O/ph.txt 2>&1 || { cat $O/ph.txt; exit 1; }
cat $O/ph.txt
