#!/bin/bash
# Shared-K/V prefill attention diagnostics (timing only, outputs wrong by design): ablib/wd4.so runs the ring and
# its barriers with no math, ablib/wd8.so the math with no copies past the prologue; against the product build.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfwgdiag
mkdir -p $O
for r in 1 2; do
  for v in prod wd4 wd8; do
    case $v in prod) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; *) L=$PWD/ablib/$v.so;; esac
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    echo "$v run $r:"; grep -E "M +(512|1024)" $O/attn_${v}_$r.txt | grep prefill
  done
done
