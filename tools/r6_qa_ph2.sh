#!/bin/bash
# Round 6: phase stamps of the fused QKV + attention launch, 7B and TinyLlama (TI_STAMP_PHASES build):
# ph1 staged, ph2 q data computed, ph3 q part reduced, ph4 k/v tiles, ph5 q gathered, ph6 attention; stream_skew col = end
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6qaph2
mkdir -p $O
for m in llama2-7b tinyllama-1.1b; do
  TI_LIB=turboinfer_amd/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py --model $m > $O/ph_$m.txt 2>&1 || { cat $O/ph_$m.txt; exit 1; }
  cat $O/ph_$m.txt
done
