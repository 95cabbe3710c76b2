#!/bin/bash
# Round-6 profile of HEAD on one box: the bench line (in-step stamped roofline), a rocprofv3 kernel trace of
# the same bench command (-> roofline_from_trace.py, kernel stats), and a FETCH_SIZE pass (-> pmc_traffic.py).
#   bash tools/r6_profile.sh <tag> [bench args...]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r6prof}; shift
O=gpurun_out/$T
mkdir -p $O
M=llama2-7b; B=1
for ((i=1; i<=$#; i++)); do a=${!i}; j=$((i+1)); [ "$a" = "--model" ] && M=${!j}; [ "$a" = "--batch" ] && B=${!j}; done
timeout -k 10 400 python3 bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench',d['value'],d['calibration']['hbm_read_GBps'],'frac',r['frac'],'span',r['span_frac'],'iso',r['isolated_frac'],r['avg_launch_us'],{k:(v['avg_us'],v['span_us']) for k,v in d['kernels'].items()})"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 64 --warmup 4 --no-cpu-baseline --kernel-reps 20 "$@" > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
DB=$(find $O/prof -name "*.db" | head -1)
if [ "$B" = "1" ]; then python3 tools/roofline_from_trace.py $DB --model $M > $O/roofline_from_trace.txt 2>&1; cat $O/roofline_from_trace.txt; fi
python3 tools/rocpd_summary.py $DB > $O/kernel_stats.txt 2>&1; head -8 $O/kernel_stats.txt
find $O/prof -name "*stats*.csv" -exec cp {} $O/ \; 2>/dev/null
rm -f $DB
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --kernel-reps 4 --stamp-steps 2 --no-cpu-baseline "$@" > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
CSV=$(find $O/pmc -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py $CSV $O/pmc_traffic.json --model $M --batch $B > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt
rm -rf $O/pmc
