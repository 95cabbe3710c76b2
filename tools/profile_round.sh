#!/bin/bash
# Round profile on the GPU box: the bench, one rocprofv3 kernel-trace pass and one FETCH_SIZE
# pass.  Summaries: tools/rocpd_summary.py, tools/roofline_from_trace.py, tools/pmc_traffic.py.
#   bash tools/profile_round.sh <tag>
# rocprofv3's kernel tracer faults (host SIGSEGV in a runtime memcpy inside hipGraphLaunch) on
# graphs instantiated after the process's first one while HIP's graph packet capture is on
# (DESIGN 5); the traced runs turn the capture off, the untraced bench keeps the default.
set -e
T=${1:-r2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
export TMPDIR=/tmp
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run -- python3 $R/bench.py --steps 64 --warmup 4 --no-cpu-baseline --kernel-reps 20 > $O/${T}_prof.log 2>&1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${T}_pmc -o run -- python3 $R/bench.py --steps 4 --warmup 2 --kernel-reps 4 --no-cpu-baseline > $O/${T}_pmc.log 2>&1
