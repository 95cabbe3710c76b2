#!/bin/bash
# The first token from the prefill's last row (TI_PREFILL_LOGITS, ti_engine_generate): engine / prefill /
# deep / C++ API / beam / serve / sampling parity, then the 512-token prefill time both ways.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pflogits
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_engine.py tests/test_gpu_prefill.py tests/test_gpu_deep.py tests/test_cpp_api.py \
  tests/test_gpu_beam.py tests/test_gpu_serve.py tests/test_gpu_sample.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  for v in 1 0; do
    TI_PREFILL_LOGITS=$v timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill_${v}_$r.txt 2>&1 || exit 1
    echo "TI_PREFILL_LOGITS=$v: $(grep 'rows 512' $O/prefill_${v}_$r.txt)"
  done
done
