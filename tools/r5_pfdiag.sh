#!/bin/bash
# Prefill attention diagnostics (TI_PF_DIAG builds, timing only -- their outputs are wrong by design):
# ablib/d1.so re-reads block 0 for every block (the math with cache-resident K / V), ablib/d2.so streams
# the K / V ring with no math; against the product build, interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfdiag
mkdir -p $O
for r in 1 2; do
  for v in prod d1 d2; do
    case $v in prod) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; *) L=$PWD/ablib/$v.so;; esac
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    echo "$v run $r:"; grep prefill $O/attn_${v}_$r.txt
  done
done
