#!/bin/bash
# Round 6: fused QKV + attention: K/V ring 3 slots issued before the GEMV (default) vs 2 slots, vs issued
# after the q part (3 / 5 slots); last-split shortening 256 keys
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/r6_ab.sh r6qa8/ab qa=.,TI_QKV_ATTN=1 kr2=turboinfer_amd/lib_kr2/libturboinfer_amd.so,TI_QKV_ATTN=1 \
  late3=turboinfer_amd/lib_late3/libturboinfer_amd.so,TI_QKV_ATTN=1 late5=turboinfer_amd/lib_late5/libturboinfer_amd.so,TI_QKV_ATTN=1 \
  x256=.,TI_QKV_ATTN=1,TI_QA_EXTRA=256 unf=.,TI_QKV_ATTN=0 -- tinyllama-1.1b || exit 1
