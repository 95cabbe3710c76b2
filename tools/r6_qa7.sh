#!/bin/bash
# Round 6: fused QKV + attention knobs: K/V ring 5 (default) vs 3 slots, last-split shortening 128 (default) / 0 / 256 keys
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/r6_ab.sh r6qa7/ab qa=.,TI_QKV_ATTN=1 kr3=turboinfer_amd/lib_kr3/libturboinfer_amd.so,TI_QKV_ATTN=1 \
  x0=.,TI_QKV_ATTN=1,TI_QA_EXTRA=0 x256=.,TI_QKV_ATTN=1,TI_QA_EXTRA=256 unf=.,TI_QKV_ATTN=0 -- tinyllama-1.1b || exit 1
