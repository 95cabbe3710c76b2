#!/bin/bash
# Batched-rows GEMM classes at 32 / 64 rows: rows kernel (default) vs the tile kernel forced down to 17 rows.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/rows_bench.py 32 64 > gpurun_out/rows_ab_rows.txt 2>&1
TI_GEMM_TILE_ROWS=17 ROWS_X=rowmajor timeout -k 10 200 python3 -u tools/rows_bench.py 32 64 > gpurun_out/rows_ab_tile.txt 2>&1
