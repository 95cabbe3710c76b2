#!/bin/bash
# Round-5 profile on the GPU box (tools/profile_round.sh + every bench configuration's PMC pass):
#   1. the default bench line (configs[2]);
#   2. one rocprofv3 --kernel-trace --stats pass of the default bench (graph packet capture off for
#      traced runs) -> kernel stats + the roofline recomputed from the trace;
#   3. one separate `--pmc FETCH_SIZE` pass per configuration (configs[1..4]) -> HBM traffic per launch.
#   bash tools/r5_profile.sh <tag>
T=${1:-r5}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
export TMPDIR=/tmp
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- \
  python3 $R/bench.py --steps 64 --warmup 4 --no-cpu-baseline --kernel-reps 20 > $O/prof.log 2>&1 || exit 1
pmc() {   # tag bench-args...
  local tag=$1; shift
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$tag -o run -- \
    python3 $R/bench.py --steps 4 --warmup 2 --kernel-reps 4 --no-cpu-baseline "$@" > $O/pmc_$tag.log 2>&1 || exit 1
}
pmc c2
pmc c1 --model tinyllama-1.1b
pmc c3 --batch 64
pmc c4 --model llama3-8b --batch 32 --kv 8192
ls -R $O | head -50
