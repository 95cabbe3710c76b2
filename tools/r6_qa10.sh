#!/bin/bash
# Round 6: fused QKV + attention at 7B / TinyLlama -- issue order: k/v-tile weights after the q part (kvwl),
# the K/V ring after the q part (kvl), both; against the default and the unfused launches
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/r6_ab.sh r6qa10/ab qa=.,TI_QKV_ATTN=1 kvwl=turboinfer_amd/lib_kvwl/libturboinfer_amd.so,TI_QKV_ATTN=1 \
  kvl=turboinfer_amd/lib_kvl/libturboinfer_amd.so,TI_QKV_ATTN=1 both=turboinfer_amd/lib_both/libturboinfer_amd.so,TI_QKV_ATTN=1 \
  unf=.,TI_QKV_ATTN=0 || exit 1
