#!/bin/bash
# Round 6: QKV + attention in one launch for one stream of TinyLlama (ti_qkv_attn_partials):
# kernel / engine parity, the TinyLlama full-depth tests, then the interleaved A/B (TI_QKV_ATTN=1 vs 0)
# and the in-step stamps of both.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6qa
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qkv_attn.py \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
grep -E "passed|failed" $O/tests.txt | tail -3
TI_QKV_ATTN=1 TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_deep.py -k "tiny or tl" \
  > $O/deep.txt 2>&1 || { tail -40 $O/deep.txt; exit 1; }
tail -3 $O/deep.txt
bash tools/r6_ab.sh r6qa/ab qa=.,TI_QKV_ATTN=1 qa0=.,TI_QKV_ATTN=1,TI_QA_EXTRA=0 unf=.,TI_QKV_ATTN=0 -- tinyllama-1.1b || exit 1
for arm in 1 0; do
  TI_QKV_ATTN=$arm timeout -k 10 180 python3 tools/stamp_probe.py --model tinyllama-1.1b > $O/stamp_$arm.txt 2>&1 || { cat $O/stamp_$arm.txt; exit 1; }
  cat $O/stamp_$arm.txt
done
