#!/bin/bash
# RECORD ONLY: the half-grid criterion was not kept (profiles/r5_prefill_wg256_ab.txt).
echo "the half-grid criterion was not kept (profiles/r5_prefill_wg256_ab.txt)"; exit 2
# 8-wave prefill attention also when its grid covers half the CUs (7B 256-row chunks): prefill-attention parity,
# then the attention alone, the previous commit's build (ablib/prev.so) against the new one, interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfwg256
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for v in prev new; do
    case $v in prev) L=$PWD/ablib/prev.so;; new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; esac
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    echo "$v run $r:"; grep prefill $O/attn_${v}_$r.txt
  done
done
