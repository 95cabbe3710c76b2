#!/bin/bash
# Round 6: fused QKV + attention, q split over the head's workgroups, exchanged in-launch; q part published before the k/v tile, split s on XCD s
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6qa6
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qkv_attn.py \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
bash tools/r6_ab.sh r6qa6/ab qa=.,TI_QKV_ATTN=1 unf=.,TI_QKV_ATTN=0 -- tinyllama-1.1b || exit 1
TI_QKV_ATTN=1 timeout -k 10 180 python3 tools/stamp_probe.py --model tinyllama-1.1b > $O/stamp_1.txt 2>&1 || { cat $O/stamp_1.txt; exit 1; }
cat $O/stamp_1.txt
TI_QKV_ATTN=1 TI_LIB=turboinfer_amd/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py --model tinyllama-1.1b > $O/ph.txt 2>&1 || { cat $O/ph.txt; exit 1; }
cat $O/ph.txt
