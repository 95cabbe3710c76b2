#!/bin/bash
# Rows-kernel grid fix (whole XCD rows): M sweep, batched tests, configs[3]/[4] lines.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batched.py tests/test_gpu_g32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rfix_tests.log 2>&1
timeout -k 10 200 python3 -u tools/rows_m_sweep.py > gpurun_out/rows_m_sweep_fix.txt 2>&1
timeout -k 10 300 python3 -u bench.py --batch 64 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rfix_c3.json 2> gpurun_out/rfix.err
timeout -k 10 300 python3 -u bench.py --model llama3-8b --batch 32 --kv 8192 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rfix_c4.json 2>> gpurun_out/rfix.err
timeout -k 10 300 python3 -u bench.py --batch 48 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rfix_b48.json 2>> gpurun_out/rfix.err
