#!/bin/bash
# Round 6: the step's own key attended inside the fused QKV + attention launch (TI_QA_NEWKEY=1, HEAD) vs merged
# by the O projection (lib_nt: TI_QA_NEWKEY=0); parity of the fused launch, the fold / engine tests it touches,
# interleaved A/B, phase stamps
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6nk
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qkv_attn.py tests/test_gpu_fold.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/r6_ab.sh r6nk/ab nk=. nt=turboinfer_amd/lib_nt/libturboinfer_amd.so unf=.,TI_QKV_ATTN=0 || exit 1
TI_LIB=turboinfer_amd/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py > $O/ph.txt 2>&1 || { cat $O/ph.txt; exit 1; }
grep -E "qkv|^o |class|B=1" $O/ph.txt
TI_LIB=turboinfer_amd/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py --model tinyllama-1.1b > $O/ph_tl.txt 2>&1 || { cat $O/ph_tl.txt; exit 1; }
grep -E "qkv|^o |class|B=1" $O/ph_tl.txt
