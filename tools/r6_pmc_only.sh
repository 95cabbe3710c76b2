#!/bin/bash
# Round 6: the FETCH_SIZE pass of tools/r6_profile.sh alone (-> pmc_traffic.py), for configs[2] or another model
#   bash tools/r6_pmc_only.sh <tag> [bench args...]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r6pmc}; shift
O=gpurun_out/$T
mkdir -p $O
M=llama2-7b; B=1
for ((i=1; i<=$#; i++)); do a=${!i}; j=$((i+1)); [ "$a" = "--model" ] && M=${!j}; [ "$a" = "--batch" ] && B=${!j}; done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --kernel-reps 4 --stamp-steps 2 --no-cpu-baseline "$@" > $O/pmc.log 2>&1 || { grep -v "^    @" $O/pmc.log | tail -5; exit 1; }
CSV=$(find $O/pmc -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py $CSV $O/pmc_traffic.json --model $M --batch $B > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt
rm -rf $O/pmc
