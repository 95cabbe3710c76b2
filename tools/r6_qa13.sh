#!/bin/bash
# Round 6: fused QKV + attention at head_dim 128 -- the k / v tiles' weights issued up front (HEAD) vs after
# staging (lib_prev = the previous commit); parity of the new order; phase stamps
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6qa13
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qkv_attn.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/r6_ab.sh r6qa13/ab qa=. prev=turboinfer_amd/lib_prev/libturboinfer_amd.so unf=.,TI_QKV_ATTN=0 || exit 1
TI_LIB=turboinfer_amd/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py > $O/ph.txt 2>&1 || { cat $O/ph.txt; exit 1; }
grep -E "qkv|class" $O/ph.txt
