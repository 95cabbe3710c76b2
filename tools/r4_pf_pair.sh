#!/bin/bash
# Prefill attention: two key blocks per online-softmax step (abx/pair) vs the product (one block),
# parity under the variant, then per-launch times and 512-token prefill, x2 interleaved.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pair
mkdir -p $O
P=$GRAFT_REPO_ROOT/abx/pair/libturboinfer_amd.so
TI_LIB=$P timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py "tests/test_gpu_deep.py::test_deep_prefill_then_decode" -x -q --timeout 150 --timeout-method thread > $O/tests.txt 2>&1
for rep in 1 2; do
  for v in base pair; do
    if [ $v = pair ]; then export TI_LIB=$P; else unset TI_LIB; fi
    echo "$v $rep" >> $O/attn.txt
    timeout -k 10 120 python3 -u tools/prefill_attn_time.py >> $O/attn.txt 2>&1
    echo "$v $rep" >> $O/prefill.txt
    timeout -k 10 200 python3 tools/prefill_bench.py 512 >> $O/prefill.txt 2>&1
  done
done
