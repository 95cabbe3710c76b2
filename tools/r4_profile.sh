#!/bin/bash
# Round-4 profile on the GPU box (tools/profile_round.sh with the persistent decode on):
# the bench line, one rocprofv3 kernel-trace + stats pass, one FETCH_SIZE pass.
#   bash tools/r4_profile.sh <tag>
set -e
T=${1:-r4}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
export TMPDIR=/tmp
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run -- python3 $R/bench.py --steps 64 --warmup 4 --no-cpu-baseline --kernel-reps 20 > $O/${T}_prof.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${T}_pmc -o run -- python3 $R/bench.py --steps 4 --warmup 2 --kernel-reps 4 --no-cpu-baseline > $O/${T}_pmc.log 2>&1
