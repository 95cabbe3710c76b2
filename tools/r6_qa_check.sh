#!/bin/bash
# Round 6: the fused QKV + attention on by default -- its parity tests, the engine / fold / kernel GPU tests
# and every full-depth TinyLlama test (TI_PARITY_LOG)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6qachk
mkdir -p $O
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_qkv_attn.py tests/test_gpu_fold.py tests/test_gpu_engine.py tests/test_gpu_deep.py -k "not llama2_7b_64 and not llama3_8b_32" \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
