#!/bin/bash
# Round 6: the fused launch's issue order -- the own generation and the rms partials out of the staging wait,
# and at head_dim 128 a barrier between the q weights' issue and the k / v weights' (HEAD = both; lib_nb = no
# barrier; lib_prev = the committed library): parity, interleaved A/B, phase stamps
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6qkvb2
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qkv_attn.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/r6_ab.sh r6qkvb2/ab qb=. nb=turboinfer_amd/lib_nb/libturboinfer_amd.so prev=turboinfer_amd/lib_prev/libturboinfer_amd.so || exit 1
TI_LIB=turboinfer_amd/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py > $O/ph.txt 2>&1 || { cat $O/ph.txt; exit 1; }
grep -E "qkv|class" $O/ph.txt
TI_LIB=turboinfer_amd/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py --model tinyllama-1.1b > $O/ph_tl.txt 2>&1 || { cat $O/ph_tl.txt; exit 1; }
grep -E "qkv|class" $O/ph_tl.txt
