#!/bin/bash
# Wide 17..64-row GEMMs on the tile kernel (TI_GEMM_TILE_WIDE_MN default | 0 off): tests, rows_bench, configs[3]/[4].
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batched.py tests/test_gpu_engine.py tests/test_gpu_deep.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wide_tests.log 2>&1
timeout -k 10 200 python3 -u tools/rows_bench.py 32 48 64 > gpurun_out/wide_on.txt 2>&1
for v in on off on off; do
  if [ $v = off ]; then export TI_GEMM_TILE_WIDE_MN=0; else unset TI_GEMM_TILE_WIDE_MN; fi
  timeout -k 10 300 python3 -u bench.py --batch 64 --steps 20 --warmup 3 --no-cpu-baseline >> gpurun_out/wide_c3_$v.jsonl 2>> gpurun_out/wide.err
  timeout -k 10 300 python3 -u bench.py --model llama3-8b --batch 32 --kv 8192 --steps 20 --warmup 3 --no-cpu-baseline >> gpurun_out/wide_c4_$v.jsonl 2>> gpurun_out/wide.err
done
