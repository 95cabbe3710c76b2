#!/bin/bash
# Round-6 final on HEAD: the whole -m gpu suite (parity log), smoke, the default bench line (with the CPU
# baseline), the side configurations (TinyLlama, 64 streams, Llama-3-8B 32 streams) and the 512-token prefill
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6final}
mkdir -p $O
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 1500 python3 -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -x > $O/gpu_suite.txt 2>&1; rc=$?
tail -3 $O/gpu_suite.txt
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $O/gpu_suite.txt | head -20; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench',d['value'],d['calibration']['hbm_read_GBps'],r['frac'],r['span_frac'],r['avg_launch_us'],d['cpu_baseline']['value'])"
: > $O/side.jsonl
for args in "--model tinyllama-1.1b" "--batch 64" "--model llama3-8b --batch 32 --kv 8192"; do
  timeout -k 10 400 python3 bench.py --no-cpu-baseline $args >> $O/side.jsonl 2> $O/side.err || { tail $O/side.err; exit 1; }
  tail -1 $O/side.jsonl | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('side',d['config']['workload'],d['value'],d['step_roofline']['frac'])"
done
timeout -k 10 300 python3 tools/prefill_bench.py > $O/prefill.txt 2>&1 || { tail $O/prefill.txt; exit 1; }
cat $O/prefill.txt
