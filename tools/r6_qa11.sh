#!/bin/bash
# Round 6: the fused QKV + attention with the K/V ring after the q part at head_dim 128: parity, the 7B and
# TinyLlama full-depth one-stream tests, then the A/B on both models and the stamps
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6qa11
mkdir -p $O
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_qkv_attn.py tests/test_gpu_deep.py -k "qkv or one_stream or bench_replay or long_llama2_7b or long_tinyllama" \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
bash tools/r6_ab.sh r6qa11/ab qa=.,TI_QKV_ATTN=1 unf=.,TI_QKV_ATTN=0 || exit 1
TI_LIB=turboinfer_amd/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py > $O/ph_7b.txt 2>&1 || { cat $O/ph_7b.txt; exit 1; }
cat $O/ph_7b.txt
