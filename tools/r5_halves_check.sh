#!/bin/bash
# The tile GEMM with TI_TILE_HALVES=1 (default): tile / prefill / g32 parity, full-depth 512-row-chunk
# prefill, the 512-token prefill time (tools/prefill_bench.py) and the tile GEMMs (tools/rows_bench.py).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/halves
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_batched.py tests/test_gpu_prefill.py tests/test_gpu_g32.py tests/test_gpu_prefill_attn.py \
  "tests/test_gpu_deep.py::test_deep_prefill_512_row_chunks" "tests/test_gpu_deep.py::test_deep_prefill_then_decode" \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill_$r.txt 2>&1 || exit 1
  cat $O/prefill_$r.txt
done
timeout -k 10 200 python3 tools/rows_bench.py 512 > $O/rows_512.txt 2>&1 || exit 1
