#!/bin/bash
# Split-K seam cost: the product build vs no merge (EXP 512) vs no read-back (EXP 1024), 32 / 64 rows.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/rows_bench.py 64 > gpurun_out/splitk_diag_prod.txt 2>&1
TI_LIB=$GRAFT_REPO_ROOT/exp/x512/libturboinfer_amd.so timeout -k 10 200 python3 -u tools/rows_bench.py 64 > gpurun_out/splitk_diag_512.txt 2>&1
TI_LIB=$GRAFT_REPO_ROOT/exp/x1024/libturboinfer_amd.so timeout -k 10 200 python3 -u tools/rows_bench.py 64 > gpurun_out/splitk_diag_1024.txt 2>&1
