#!/bin/bash
# Tile GEMM bottleneck split (512 rows): product vs no compute (EXP 2048) vs no weight stream
# (EXP 4096: re-reads of the first group) vs no activation stream (EXP 8192).
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/rows_bench.py 512 > gpurun_out/tdiag_prod.txt 2>&1
for X in 2048 4096 8192; do
  TI_LIB=$GRAFT_REPO_ROOT/exp/x$X/libturboinfer_amd.so timeout -k 10 200 python3 -u tools/rows_bench.py 512 > gpurun_out/tdiag_$X.txt 2>&1
done
