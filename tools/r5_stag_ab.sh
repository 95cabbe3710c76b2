#!/bin/bash
# RECORD ONLY: TI_TILE_STAG was removed after these A/Bs (profiles/r5_tile_stagger_ab.txt, r5_tile_halves_ab.txt);
# the halves they isolated are the default now (TI_TILE_HALVES).  The script stops here.
echo "TI_TILE_STAG was removed (profiles/r5_tile_stagger_ab.txt)"; exit 2
# Staggered tile GEMM (TI_TILE_STAG=1 build in tools/bin/stag/): parity (tile / prefill tests with
# the variant library), then tools/rows_bench.py at 256 / 512 / 1024 rows and the 512-token
# prefill, interleaved per arm.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/stag
mkdir -p $O
S=$GRAFT_REPO_ROOT/tools/bin/stag/libturboinfer_amd.so
TI_LIB=$S timeout -k 10 500 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_batched.py tests/test_gpu_prefill.py "tests/test_gpu_deep.py::test_deep_prefill_512_row_chunks" \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  for arm in base stag; do
    L=""; [ $arm = stag ] && L=$S
    TI_LIB=$L timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > $O/rows_${arm}_$r.txt 2>&1 || exit 1
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill_${arm}_$r.txt 2>&1 || exit 1
    echo "== $arm $r"; grep -E "M= 512|M=512" $O/rows_${arm}_$r.txt | head -8; head -2 $O/prefill_${arm}_$r.txt
  done
done
