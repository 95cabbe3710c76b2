#!/bin/bash
# Round 6: the fused launch's bounded waits -- the lost-sibling test and the rest of the fused launch's parity
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6fault
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qkv_attn.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
grep -E "passed|failed|PASS|FAIL" $O/tests.txt | tail -20
