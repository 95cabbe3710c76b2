#!/bin/bash
# Last-row logits for several equal-length streams: engine / prefill / deep / C++ API / beam / serve / sampling parity.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pflogits2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_engine.py tests/test_gpu_prefill.py tests/test_gpu_deep.py tests/test_cpp_api.py \
  tests/test_gpu_beam.py tests/test_gpu_serve.py tests/test_gpu_sample.py tests/test_gpu_threads.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
