#!/bin/bash
# The bench line of configs[2] (default) and of the side configs [1], [3], [4] on one box.
#   bash tools/side_configs.sh <tag>     -> gpurun_out/<tag>_side.jsonl
set -e
T=${1:-r3}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
export TMPDIR=/tmp
mkdir -p $O
cd $R
: > $O/${T}_side.jsonl
timeout -k 10 300 python3 bench.py --no-cpu-baseline >> $O/${T}_side.jsonl 2> $O/${T}_side_c2.err
timeout -k 10 300 python3 bench.py --model tinyllama-1.1b --no-cpu-baseline >> $O/${T}_side.jsonl 2> $O/${T}_side_c1.err
timeout -k 10 300 python3 bench.py --batch 64 --steps 32 --warmup 4 --no-cpu-baseline >> $O/${T}_side.jsonl 2> $O/${T}_side_c3.err
timeout -k 10 300 python3 bench.py --model llama3-8b --batch 32 --kv 8192 --steps 32 --warmup 4 --no-cpu-baseline >> $O/${T}_side.jsonl 2> $O/${T}_side_c4.err
