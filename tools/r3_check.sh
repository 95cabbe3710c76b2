#!/bin/bash
# Round-3 GPU check: the full-depth parity tests (errors logged) and the round's new tests, then
# the bench side configs.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
export TMPDIR=/tmp
mkdir -p $O
cd $R
rm -f $O/deep_parity.jsonl
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 500 python3 -u -m pytest tests/test_gpu_deep.py tests/test_gpu_threads.py tests/test_gpu_beam.py -v --timeout 200 --timeout-method thread > $O/deep_tests.log 2>&1 || true
bash tools/side_configs.sh ${1:-r3start}
