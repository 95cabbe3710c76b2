#!/bin/bash
# Split-K tile GEMM (under-filled grids only): batched kernel + prefill tests, rows_bench at
# 65..512 rows with / without split-K, prefill bench with / without.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batched.py tests/test_gpu_prefill.py -x -v --timeout 120 --timeout-method thread > gpurun_out/splitk_tests.log 2>&1
timeout -k 10 200 python3 -u tools/rows_bench.py 65 128 512 > gpurun_out/splitk_rows_on.txt 2>&1
TI_GEMM_SPLITK=0 timeout -k 10 200 python3 -u tools/rows_bench.py 65 128 512 > gpurun_out/splitk_rows_off.txt 2>&1
timeout -k 10 200 python3 -u tools/prefill_bench.py 512 > gpurun_out/splitk_prefill_on.txt 2>&1
TI_GEMM_SPLITK=0 timeout -k 10 200 python3 -u tools/prefill_bench.py 512 > gpurun_out/splitk_prefill_off.txt 2>&1
