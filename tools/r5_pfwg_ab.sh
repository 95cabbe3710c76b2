#!/bin/bash
# Prefill attention with each kv-head's K / V blocks shared in LDS by a workgroup of 4 query blocks
# (attn_prefill_wg_kernel: TI_PF_WG=2 eight waves in key-split halves, 1 four waves) against the per-wave kernel
# (TI_PF_WG=0): parity every way, then
# the attention alone and the 512-token prefill, interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfwg
mkdir -p $O
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in 1 0; do
  TI_PF_WG=$v timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_prefill_attn.py > $O/tests$v.txt 2>&1 || { tail -40 $O/tests$v.txt; exit 1; }
  tail -1 $O/tests$v.txt
done
for r in 1 2; do
  for v in 2 1 0; do
    TI_PF_WG=$v timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    TI_PF_WG=$v timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill_${v}_$r.txt 2>&1 || exit 1
    echo "TI_PF_WG=$v run $r: $(grep 'rows 512' $O/prefill_${v}_$r.txt)"
    grep prefill $O/attn_${v}_$r.txt
  done
done
