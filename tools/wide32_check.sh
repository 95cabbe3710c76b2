#!/bin/bash
# 17..32-row wide outputs on the tile kernel (TI_GEMM_TILE_WIDE_N32): parity tests, then 7B bench
# lines at 24 and 32 streams against TI_GEMM_TILE_WIDE_N32=0 (the rows x N >= 850000 rule alone).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batched.py tests/test_gpu_deep.py tests/test_gpu_engine.py tests/test_gpu_serve.py > gpurun_out/w32_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/w32_tests.txt; exit 1; }
: > gpurun_out/w32.jsonl
for r in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export TI_GEMM_TILE_WIDE_N32=0; else unset TI_GEMM_TILE_WIDE_N32; fi
    for b in 24 32; do
      timeout -k 10 200 python3 bench.py --batch $b --steps 32 --warmup 4 --no-cpu-baseline | sed "s/^/$v b$b /" >> gpurun_out/w32.jsonl || exit 1
    done
  done
done
