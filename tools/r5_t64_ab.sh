#!/bin/bash
# RECORD ONLY: TI_TILE_ROWS was removed after this A/B (profiles/r5_tile64_ab.txt); the script stops here.
echo "TI_TILE_ROWS was removed (profiles/r5_tile64_ab.txt)"; exit 2
# 64-row GEMMs on the tile kernel (TI_TILE_ROWS=49 build in tools/bin/t64/: split-K tile GEMM, row-major
# operands, no batched fold) vs the batched-rows kernel: tools/rows_bench.py 64 and the configs[3] bench line.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/t64
mkdir -p $O
S=$GRAFT_REPO_ROOT/tools/bin/t64/libturboinfer_amd.so
TI_LIB=$S timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_engine.py -k "64_streams or batch" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for arm in base t64; do
    L=""; [ $arm = t64 ] && L=$S
    TI_LIB=$L timeout -k 10 200 python3 tools/rows_bench.py 64 > $O/rows_${arm}_$r.txt 2>&1 || exit 1
    TI_LIB=$L timeout -k 10 300 python3 bench.py --batch 64 --steps 16 --warmup 3 --no-cpu-baseline > $O/c3_${arm}_$r.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$O/c3_${arm}_$r.json'));print('c3 $arm $r', d['value'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
  done
done
