#!/bin/bash
# Prefill attention: the deep K/V ring when every wave has a SIMD to itself (product: 8 blocks;
# abx/rd6: 6; abx/rd3: 3 = the round-3 kernel), parity then per-launch times and 512-token
# prefill, interleaved on one box.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfd
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py "tests/test_gpu_deep.py::test_deep_prefill_then_decode" -x -q --timeout 150 --timeout-method thread > $O/tests.txt 2>&1
for rep in 1 2; do
  for v in rd3 rd6 rd8; do
    if [ $v = rd8 ]; then unset TI_LIB; else export TI_LIB=$GRAFT_REPO_ROOT/abx/$v/libturboinfer_amd.so; fi
    echo "$v $rep" >> $O/attn.txt
    timeout -k 10 120 python3 -u tools/prefill_attn_time.py >> $O/attn.txt 2>&1
    echo "$v $rep" >> $O/prefill.txt
    timeout -k 10 200 python3 tools/prefill_bench.py 512 >> $O/prefill.txt 2>&1
  done
done
