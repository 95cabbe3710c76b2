#!/bin/bash
# RECORD ONLY: kept (profiles/r5_prefill_perwave_permlane_ab.txt).
echo "kept (profiles/r5_prefill_perwave_permlane_ab.txt)"; exit 2
# The per-wave prefill attention (256-row 7B chunks, head_dim 64) with the cross-row max on v_permlane16/32_swap instead of two
# ds_bpermute round trips: prefill-attention / prefill / deep parity, then the attention alone, the previous
# commit's build (ablib/prev.so) against the new one, interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfperm2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py \
  tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for v in prev new; do
    case $v in prev) L=$PWD/ablib/prev.so;; new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; esac
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    echo "$v run $r:"; grep -E "M +(128|256)" $O/attn_${v}_$r.txt | grep prefill
  done
done
