#!/bin/bash
# 8-wave shared-K/V prefill attention: LDS ring of 8 / 12 (default) / 16 blocks (1 / 2 / 3 iterations of DMA ahead).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfring2
mkdir -p $O
for v in r8 r16; do
  TI_LIB=$PWD/ablib/$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefill_attn.py \
    > $O/tests_$v.txt 2>&1 || { tail -30 $O/tests_$v.txt; exit 1; }
  tail -1 $O/tests_$v.txt
done
for r in 1 2; do
  for v in new r8 r16; do
    case $v in new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; *) L=$PWD/ablib/$v.so;; esac
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    echo "$v run $r:"; grep -E "M +(512|1024)" $O/attn_${v}_$r.txt | grep prefill
  done
done
