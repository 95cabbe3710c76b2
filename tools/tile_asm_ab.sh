#!/bin/bash
# Prefill tile GEMM: activation DMA issued from inline asm (default build) vs the builtin DMA
# (exp/tile0, TI_TILE_ASM=0).  Parity first, then per-shape timing and the 512-token prefill.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batched.py tests/test_gpu_prefill.py tests/test_gpu_g32.py tests/test_gpu_prefill_attn.py tests/test_gpu_sample.py -q -k "not sampled_generate or 9000" --timeout 120 --timeout-method thread > gpurun_out/tile_tests.log 2>&1
timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > gpurun_out/tile_asm_rows.txt 2>&1
TI_LIB=$GRAFT_REPO_ROOT/exp/tile0/libturboinfer_amd.so timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > gpurun_out/tile_old_rows.txt 2>&1
timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/tile_asm_prefill.txt 2>&1
TI_LIB=$GRAFT_REPO_ROOT/exp/tile0/libturboinfer_amd.so timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/tile_old_prefill.txt 2>&1
