#!/bin/bash
# Batched-rows kernel with row blocks split over workgroups: batched + engine tests, rows_bench A/B,
# and the configs[3] / [4] bench lines.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batched.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rsplit_tests.log 2>&1
timeout -k 10 200 python3 -u tools/rows_bench.py 32 64 > gpurun_out/rsplit_on.txt 2>&1
TI_GEMM_ROWS_SPLIT=0 timeout -k 10 200 python3 -u tools/rows_bench.py 32 64 > gpurun_out/rsplit_off.txt 2>&1
timeout -k 10 300 python3 -u bench.py --model llama2-7b --batch 64 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rsplit_c3_on.json 2> gpurun_out/rsplit_c3.err
TI_GEMM_ROWS_SPLIT=0 timeout -k 10 300 python3 -u bench.py --model llama2-7b --batch 64 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rsplit_c3_off.json 2>> gpurun_out/rsplit_c3.err
timeout -k 10 300 python3 -u bench.py --model llama3-8b --batch 32 --kv 8192 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rsplit_c4_on.json 2>> gpurun_out/rsplit_c3.err
TI_GEMM_ROWS_SPLIT=0 timeout -k 10 300 python3 -u bench.py --model llama3-8b --batch 32 --kv 8192 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rsplit_c4_off.json 2>> gpurun_out/rsplit_c3.err
