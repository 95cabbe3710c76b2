#!/bin/bash
# RECORD ONLY: TI_PF_WG_LATE_DMA stays 0 (profiles/r5_prefill_wg_latedma_ab.txt).
echo "TI_PF_WG_LATE_DMA stays 0 (profiles/r5_prefill_wg_latedma_ab.txt)"; exit 2
# 8-wave shared-K/V prefill attention: the next DMAs issued after the step's S = K Q^T (ablib/late.so) vs before it.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pflate
mkdir -p $O
for v in late; do
  TI_LIB=$PWD/ablib/$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefill_attn.py \
    > $O/tests_$v.txt 2>&1 || { tail -30 $O/tests_$v.txt; exit 1; }
  tail -1 $O/tests_$v.txt
done
for r in 1 2; do
  for v in new late; do
    case $v in new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; *) L=$PWD/ablib/$v.so;; esac
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    echo "$v run $r:"; grep -E "M +(512|1024)" $O/attn_${v}_$r.txt | grep prefill
  done
done
