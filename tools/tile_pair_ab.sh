#!/bin/bash
# Tile GEMM: one barrier per pair of groups (TI_TILE_PAIR=1, product) vs one barrier per group
# (exp/pair0): parity, phase split (tools/probe_tile), per-shape timing, prefill.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pair
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batched.py tests/test_gpu_g32.py tests/test_gpu_prefill.py tests/test_gpu_prefill_attn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pair/tests.log 2>&1
timeout -k 10 120 ./tools/probe_tile > gpurun_out/pair/probe.txt 2>&1
for i in 1 2; do
  timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/pair/prefill_on$i.txt 2>&1
  TI_LIB=$GRAFT_REPO_ROOT/exp/pair0/libturboinfer_amd.so timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/pair/prefill_off$i.txt 2>&1
done
timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > gpurun_out/pair/rows_on.txt 2>&1
