#!/bin/bash
# Stop token and the prefill's first token: engine / C++ API / beam / serve parity.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/stop0
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_engine.py tests/test_cpp_api.py tests/test_gpu_beam.py tests/test_gpu_serve.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
