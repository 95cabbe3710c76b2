#!/bin/bash
# Prefill attention parity with every kernel forced (ti_attn_prefill_set_kernel) plus the prefill / deep suites.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfkern
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { grep -E "FAILED|Error|error" $O/tests.txt | head -30; tail -30 $O/tests.txt; exit 1; }
grep -E "passed|failed" $O/tests.txt | tail -2
