#!/bin/bash
# Tile-kernel LDS swizzle for the ds_read_b128 lane groups (TI_TILE_SWZ4=1, default) vs the row & 15 swizzle
# (tools/bin/swz0/): parity, SQ_LDS_BANK_CONFLICT on the 7B QKV at 512 rows, tile GEMMs and the 512-token prefill.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/swz
mkdir -p $O
S0=$GRAFT_REPO_ROOT/tools/bin/swz0/libturboinfer_amd.so
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_batched.py \
  tests/test_gpu_g32.py tests/test_gpu_prefill.py tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for arm in swz4 swz0; do
  L=""; [ $arm = swz0 ] && L=$S0
  TI_LIB=$L timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES --output-format csv \
    -d $O/pmc_$arm -o t -- python3 tools/tile_one.py > $O/pmc_$arm.log 2>&1 || exit 1
done
for r in 1 2; do
  for arm in swz4 swz0; do
    L=""; [ $arm = swz0 ] && L=$S0
    TI_LIB=$L timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > $O/rows_${arm}_$r.txt 2>&1 || exit 1
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill_${arm}_$r.txt 2>&1 || exit 1
    echo "$arm run $r: $(grep 'rows 512' $O/prefill_${arm}_$r.txt)"
  done
done
