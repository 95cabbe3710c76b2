#!/bin/bash
# configs[4] attention: long-range GQA K/V ring depth (TI_ATTN_RING_LONG 4 product | 6 | 8 in exp/).
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/c4_ring_ab.txt
for v in 4 6 8 4; do
  if [ $v = 4 ]; then L=""; else L=$GRAFT_REPO_ROOT/exp/l$v/libturboinfer_amd.so; fi
  TI_LIB=$L timeout -k 10 300 python3 -u bench.py --model llama3-8b --batch 32 --kv 8192 --steps 16 --warmup 3 --no-cpu-baseline > gpurun_out/c4_r$v.json 2>> gpurun_out/c4_ring_ab.err
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/c4_r$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('attention'))")" >> gpurun_out/c4_ring_ab.txt
done
TI_LIB=$GRAFT_REPO_ROOT/exp/l6/libturboinfer_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_engine.py -x -q -k "llama3 or 8192" --timeout 200 --timeout-method thread > gpurun_out/c4_ring_tests.log 2>&1
