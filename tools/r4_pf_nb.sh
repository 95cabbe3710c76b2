#!/bin/bash
# Prefill attention: 4 key blocks per softmax step on the deep ring (abx/nb4) and a 2-deep paired
# ring for chunks beyond one wave per SIMD (abx/r2) vs the product; parity under each variant,
# then per-launch times and 512-token prefill, x2 interleaved.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/nb
mkdir -p $O
for v in nb4 r2; do
  TI_LIB=$GRAFT_REPO_ROOT/abx/$v/libturboinfer_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py "tests/test_gpu_deep.py::test_deep_prefill_then_decode" -x -q --timeout 150 --timeout-method thread > $O/tests_$v.txt 2>&1
done
for rep in 1 2; do
  for v in base nb4 r2; do
    if [ $v = base ]; then unset TI_LIB; else export TI_LIB=$GRAFT_REPO_ROOT/abx/$v/libturboinfer_amd.so; fi
    echo "$v $rep" >> $O/attn.txt
    timeout -k 10 120 python3 -u tools/prefill_attn_time.py >> $O/attn.txt 2>&1
    echo "$v $rep" >> $O/prefill.txt
    timeout -k 10 200 python3 tools/prefill_bench.py 512 >> $O/prefill.txt 2>&1
  done
done
