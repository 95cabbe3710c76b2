#!/bin/bash
# Prefill attention with the K / V ring kept in flight (buffer loads, unconditional refills, step order
# pinned, prologue drained): parity on the new build, then ti_attn_prefill alone and the 512-token
# prefill for the round-5 build (ablib/old.so), the new default (ring 4, pairs), ring 8 in steps of 4 blocks
# (ablib/r8.so) and ring 4 in one step of 4 (ablib/r44.so), interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfring
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in r8 r44; do
  TI_LIB=$PWD/ablib/$v.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_prefill_attn.py > $O/tests_$v.txt 2>&1 || { tail -40 $O/tests_$v.txt; exit 1; }
  tail -1 $O/tests_$v.txt
done
for r in 1 2; do
  for v in old new r8 r44; do
    case $v in old) L=$PWD/ablib/old.so;; new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; r8) L=$PWD/ablib/r8.so;; r44) L=$PWD/ablib/r44.so;; esac
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill_${v}_$r.txt 2>&1 || exit 1
    echo "$v run $r: $(grep 'rows 512' $O/prefill_${v}_$r.txt)"
    grep prefill $O/attn_${v}_$r.txt
  done
done
