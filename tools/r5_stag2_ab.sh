#!/bin/bash
# RECORD ONLY: TI_TILE_STAG was removed after these A/Bs (profiles/r5_tile_stagger_ab.txt, r5_tile_halves_ab.txt);
# the halves they isolated are the default now (TI_TILE_HALVES).  The script stops here.
echo "TI_TILE_STAG was removed (profiles/r5_tile_stagger_ab.txt)"; exit 2
# Decomposes the stagger A/B (profiles/r5_tile_stagger_ab.txt): TI_TILE_STAG=2 runs the staggered
# loop's issue order (activations 2 groups ahead, halves back to back) with no wave late; TI_TILE_HALVES=1
# the halves in the product loops (activations 3 groups ahead).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/stag2h
mkdir -p $O
for r in 1 2; do
  for arm in base stag2 halves; do
    L=""; [ $arm != base ] && L=$GRAFT_REPO_ROOT/tools/bin/$arm/libturboinfer_amd.so
    TI_LIB=$L timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > $O/rows_${arm}_$r.txt 2>&1 || exit 1
    echo "== $arm $r"; grep -E "7b qkv|7b gate_up|l3 qkv" $O/rows_${arm}_$r.txt | head -3
  done
done
