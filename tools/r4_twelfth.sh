#!/bin/bash
# Persistent decode: what the hand-off waits cost. Phase timelines of the product, of gathers that take
# what they find (no tag waits, pnw, garbage results) and of that without GEMV math (pnwnm).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in base pnw pnwnm; do
  L=""; [ $v = base ] || L=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so
  TI_PDS=1 TI_PDS_TS=1 TI_LIB=$L timeout -k 10 200 python3 -u tools/pds_phases.py > gpurun_out/r4l_phases_$v.txt 2>&1 || exit 1
done
echo "done12"
