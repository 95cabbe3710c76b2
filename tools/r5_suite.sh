#!/bin/bash
# Round-5 GPU check: the whole -m gpu suite (parity log), smoke, the default bench line.
#   bash tools/r5_suite.sh <tag>
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r5}
O=gpurun_out/$T
mkdir -p $O
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread --durations=20 > $O/gpu_suite.txt 2>&1
rc=$?
echo "suite rc=$rc" >> $O/gpu_suite.txt
tail -5 $O/gpu_suite.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
