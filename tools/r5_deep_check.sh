#!/bin/bash
# Full-depth parity (tests/test_gpu_deep.py, incl. the 640-token prompt at 512- and 1024-row chunk limits).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/deep
mkdir -p $O
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 600 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
