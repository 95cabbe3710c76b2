#!/bin/bash
# RECORD ONLY: the prompt-chunk fold was reverted after this A/B (profiles/r5_prefill_fold_ab.txt); the script stops here.
echo "TI_PREFILL_FOLD was reverted (profiles/r5_prefill_fold_ab.txt)"; exit 2
# Prompt-chunk fold (TI_PREFILL_FOLD, tile-kernel fold producer): fold / tile / prefill / deep / engine parity,
# then the 512-token prefill both ways, interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pffold
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_batched.py tests/test_gpu_fold.py tests/test_gpu_prefill.py tests/test_gpu_deep.py tests/test_gpu_engine.py \
  tests/test_cpp_api.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do
  for v in 1 0; do
    TI_PREFILL_FOLD=$v timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill_${v}_$r.txt 2>&1 || exit 1
    echo "TI_PREFILL_FOLD=$v: $(grep 'rows 512' $O/prefill_${v}_$r.txt)"
  done
done
