#!/bin/bash
# RECORD ONLY: TI_PF_WPB was not kept (profiles/r5_prefill_attn_wpb_ab.txt); the script stops here.
echo "TI_PF_WPB was not kept (profiles/r5_prefill_attn_wpb_ab.txt)"; exit 2
# Prefill attention: query blocks of one kv-head co-located in one workgroup (TI_PF_WPB 2 / 4 builds in
# tools/bin/wpb*/) vs one wave per workgroup: parity with the variant, the attention alone and the
# 512-token prefill, interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/wpb
mkdir -p $O
TI_LIB=$GRAFT_REPO_ROOT/tools/bin/wpb4/libturboinfer_amd.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 250 \
  --timeout-method thread tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for arm in base wpb2 wpb4; do
    L=""; [ $arm != base ] && L=$GRAFT_REPO_ROOT/tools/bin/$arm/libturboinfer_amd.so
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${arm}_$r.txt 2>&1 || exit 1
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill_${arm}_$r.txt 2>&1 || exit 1
    echo "$arm run $r: $(grep 'rows 512' $O/prefill_${arm}_$r.txt)"
    grep prefill $O/attn_${arm}_$r.txt
  done
done
