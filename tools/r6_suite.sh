#!/bin/bash
# Round-6 full GPU suite + smoke + default bench + trace, outputs under gpurun_out/<tag>
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r6suite}
O=gpurun_out/$T
mkdir -p $O
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 1500 python3 -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -x > $O/gpu_suite.txt 2>&1; rc=$?
tail -3 $O/gpu_suite.txt
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $O/gpu_suite.txt | head -20; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench',d['value'],d['calibration']['hbm_read_GBps'],r['frac'],r['span_frac'],r['avg_launch_us'],d['cpu_baseline']['value'])"
