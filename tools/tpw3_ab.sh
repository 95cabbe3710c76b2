#!/bin/bash
# Tile GEMM with 3 weight tiles per wave (192-column workgroups) vs without (TI_TILE_TPW3=0):
# parity of the batched / group-32 / prefill paths, then per-shape timing and the 512-token prefill.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tpw3
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batched.py tests/test_gpu_g32.py tests/test_gpu_prefill.py -q -x --timeout 120 --timeout-method thread > gpurun_out/tpw3/tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > gpurun_out/tpw3/rows_on$i.txt 2>&1
  TI_TILE_TPW3=0 timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > gpurun_out/tpw3/rows_off$i.txt 2>&1
  timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/tpw3/prefill_on$i.txt 2>&1
  TI_TILE_TPW3=0 timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/tpw3/prefill_off$i.txt 2>&1
done
