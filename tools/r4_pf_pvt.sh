#!/bin/bash
# Prefill attention with O^T = V^T P^T (alpha in place, no per-block broadcast) and clamped V rows
# (no branch per load): parity, then per-launch times and 512-token prefill against the previous
# commit's build (abx/prev) and the same code with a 4-deep ring (abx/r4), x2.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pvt
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py "tests/test_gpu_deep.py::test_deep_prefill_then_decode" -x -q --timeout 150 --timeout-method thread > $O/tests.txt 2>&1
for rep in 1 2; do
  for v in prev r4 pvt; do
    if [ $v = pvt ]; then unset TI_LIB; else export TI_LIB=$GRAFT_REPO_ROOT/abx/$v/libturboinfer_amd.so; fi
    echo "$v $rep" >> $O/attn.txt
    timeout -k 10 120 python3 -u tools/prefill_attn_time.py >> $O/attn.txt 2>&1
    echo "$v $rep" >> $O/prefill.txt
    timeout -k 10 200 python3 tools/prefill_bench.py 512 >> $O/prefill.txt 2>&1
  done
done
