#!/bin/bash
# RECORD ONLY: TI_PF_SPLIT was reverted after this A/B (profiles/r5_prefill_attn_split_ab.txt); the script stops here.
echo "TI_PF_SPLIT was reverted (profiles/r5_prefill_attn_split_ab.txt)"; exit 2
# Two-wave key split of the prefill attention (TI_PF_SPLIT): kernel / prefill / deep parity, the attention
# alone at 256 / 512 / 1024 rows and the 512-token prefill, TI_PF_SPLIT=1 / 0 interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfsplit
mkdir -p $O
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 600 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for v in 1 0; do
    TI_PF_SPLIT=$v timeout -k 10 200 python3 tools/prefill_attn_time.py > $O/attn_${v}_$r.txt 2>&1 || exit 1
    TI_PF_SPLIT=$v timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill_${v}_$r.txt 2>&1 || exit 1
    echo "TI_PF_SPLIT=$v run $r: $(grep 'rows 512' $O/prefill_${v}_$r.txt)"
    grep prefill $O/attn_${v}_$r.txt
  done
done
