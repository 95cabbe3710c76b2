#!/bin/bash
# Tile GEMM 32-row waves (RB 2) at <= 32 rows: parity tests, then the wide shapes at 32 rows and the
# configs[4] bench line, each against TI_TILE_RB2=0 (64-row waves) on the same box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batched.py tests/test_gpu_deep.py > gpurun_out/rb2_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/rb2_tests.txt; exit 1; }
ROWS_X=rowmajor timeout -k 10 200 python3 -u tools/rows_bench.py 17 24 32 > gpurun_out/rb2_rows.txt 2>&1 || exit 1
ROWS_X=rowmajor TI_TILE_RB2=0 timeout -k 10 200 python3 -u tools/rows_bench.py 17 24 32 > gpurun_out/rb2_rows_off.txt 2>&1 || exit 1
: > gpurun_out/rb2_c4.jsonl
for r in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export TI_TILE_RB2=0; else unset TI_TILE_RB2; fi
    timeout -k 10 200 python3 bench.py --model llama3-8b --batch 32 --kv 8192 --steps 32 --warmup 4 --no-cpu-baseline | sed "s/^/$v c4 /" >> gpurun_out/rb2_c4.jsonl || exit 1
  done
done
