#!/bin/bash
# Batched-decode GEMM bottleneck split at 32 / 64 rows (configs[4] / [3]): product vs diagnostic
# builds (make BUILD=build_xN LIB=exp/xN/libturboinfer_amd.so EXTRA=-DTI_GEMV_EXP=N):
#   rows kernel: 128 no weight stream after the first ring, 256 no activation stream;
#   tile kernel: 2048 no compute, 4096 no weight stream, 8192 no activation stream.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/rows_bench.py 32 64 > gpurun_out/rdiag_prod.txt 2>&1
for X in 128 256 2048 4096 8192; do
  TI_LIB=$GRAFT_REPO_ROOT/exp/x$X/libturboinfer_amd.so timeout -k 10 200 python3 -u tools/rows_bench.py 32 64 > gpurun_out/rdiag_$X.txt 2>&1
done
