#!/bin/bash
# TinyLlama (configs[1]) A/B: single-stream GQA attention as 8 long splits merged by the O
# projection (default) vs the round-2 policy (32 short splits, last-arriver merge).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
export TMPDIR=/tmp
mkdir -p $O
cd $R
: > $O/tl_ab.jsonl
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --model tinyllama-1.1b --no-cpu-baseline >> $O/tl_ab.jsonl 2>> $O/tl_ab.err
  TI_ATTN_GQA_PART=0 timeout -k 10 200 python3 bench.py --model tinyllama-1.1b --no-cpu-baseline >> $O/tl_ab.jsonl 2>> $O/tl_ab.err
done
TI_PARITY_LOG=$O/deep_parity_tl.jsonl timeout -k 10 300 python3 -u -m pytest tests/test_gpu_deep.py tests/test_gpu_fold.py tests/test_gpu_engine.py -k "tinyllama or fold" -v --timeout 200 --timeout-method thread > $O/tl_deep.log 2>&1
