#!/bin/bash
# RECORD ONLY: TI_PF_QK_SPLIT stays 0 (profiles/r5_prefill_wg_qksplit_ab.txt).
echo "TI_PF_QK_SPLIT stays 0 (profiles/r5_prefill_wg_qksplit_ab.txt)"; exit 2
# Shared-K/V prefill attention with S = K Q^T's hi and lo products in separate MFMA chains (TI_PF_QK_SPLIT=1,
# ablib/qks.so): parity of that build, then the attention alone against the product build, interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfqks
mkdir -p $O
TI_LIB=$PWD/ablib/qks.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py \
  tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for v in new qks; do
    case $v in qks) L=$PWD/ablib/qks.so;; new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; esac
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    echo "$v run $r:"; grep -E "M +(512|1024)" $O/attn_${v}_$r.txt | grep prefill
  done
done
