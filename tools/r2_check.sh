#!/bin/bash
# Round-2 GPU check: gpu tests, the bench, a kernel-trace profile of the bench, and the sampled
# decode under the tracer.  Every GPU step has its own time limit; steps
# chained with && so the first failure ends the call.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
export TMPDIR=/tmp
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_stats -o run -- python3 $R/bench.py --steps 64 --warmup 4 --no-cpu-baseline > $O/prof_stats.log 2>&1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_samp -o run -- python3 $R/tools/sample_bench.py 64 > $O/prof_samp.log 2>&1
