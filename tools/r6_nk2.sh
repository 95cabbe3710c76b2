#!/bin/bash
# Round 6: the fused launch with the in-launch new key as the only form (NT merge removed): the GPU tests it touches
# (fused vs unfused launches, twin engines, fold, engine, deep full-depth one-stream parity), then a bench line
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6nk2
mkdir -p $O
export TI_PARITY_LOG=$O/deep_parity.jsonl
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qkv_attn.py tests/test_gpu_fold.py tests/test_gpu_engine.py tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['calibration']['hbm_read_GBps'])"
