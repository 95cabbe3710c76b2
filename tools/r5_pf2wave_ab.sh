#!/bin/bash
# The shallow-ring prefill attention (chunks past 512 rows on 7B) held to 256 registers, two waves per SIMD:
# parity, then ti_attn_prefill alone for the previous commit's build (ablib/prev.so) and the new one, interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pf2w
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for v in prev new; do
    case $v in prev) L=$PWD/ablib/prev.so;; new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; esac
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    echo "$v run $r:"; grep prefill $O/attn_${v}_$r.txt
  done
done
