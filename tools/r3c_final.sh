#!/bin/bash
# End-of-session check: smoke, the whole GPU suite, then the bench lines of configs[2] and the side configs.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.txt 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/fin_smoke.txt; exit 1; }
timeout -k 10 780 python3 -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fin_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/fin_tests.txt; exit 1; }
bash tools/side_configs.sh fin
