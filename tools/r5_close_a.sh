#!/bin/bash
# Round-5 close, part A: the whole GPU suite (full-depth parity logged) and smoke() on the committed build.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/close
mkdir -p $O
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread \
  > $O/gpu_suite_full.txt 2>&1 || { tail -60 $O/gpu_suite_full.txt; exit 1; }
grep -E "passed|failed|skipped" $O/gpu_suite_full.txt | tail -3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -30 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
