#!/bin/bash
# Round 6: the in-step launch timeline (ti_engine_stamp_steps) and the bench's in-step roofline against
# a rocprofv3 kernel trace of the same build on the same box.
#   1-2. wave-0 phase marks (TI_STAMP_PHASES build, turboinfer_amd/lib_ph) for configs[2] and configs[1]
#   3.   bench.py (product library): roofline from in-step periods
#   4.   rocprofv3 --kernel-trace --stats of the same bench command -> roofline_from_trace.py
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6stamp
mkdir -p $O
PH=$GRAFT_REPO_ROOT/turboinfer_amd/lib_ph/libturboinfer_amd.so
TI_LIB=$PH timeout -k 10 180 python3 tools/stamp_probe.py --json $O/ph_7b.json > $O/ph_7b.txt 2>&1 || { cat $O/ph_7b.txt; exit 1; }
cat $O/ph_7b.txt
TI_LIB=$PH timeout -k 10 180 python3 tools/stamp_probe.py --model tinyllama-1.1b --json $O/ph_tl.json > $O/ph_tl.txt 2>&1 || { cat $O/ph_tl.txt; exit 1; }
cat $O/ph_tl.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench',d['value'],r['frac'],r['span_frac'],r['isolated_frac'],r['avg_launch_us'],{k:(v['avg_us'],v['span_us'],v['isolated_us']) for k,v in d['kernels'].items()})"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 64 --warmup 4 --no-cpu-baseline --kernel-reps 20 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
DB=$(find $O/prof -name "*.db" | head -1)
python3 tools/roofline_from_trace.py $DB > $O/roofline_from_trace.txt 2>&1; cat $O/roofline_from_trace.txt
python3 tools/rocpd_summary.py $DB > $O/kernel_stats.txt 2>&1; head -12 $O/kernel_stats.txt
grep -h '"frac"' $O/prof.log | head -2 || true
