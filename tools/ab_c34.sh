#!/bin/bash
# Interleaved A/B of configs[3] / [4] bench lines: exp/base (a build of the previous commit:
#   git worktree add /tmp/base HEAD && make -C /tmp/base LIB=$PWD/exp/base/libturboinfer_amd.so) vs the tree's library.
#   bash tools/ab_c34.sh <tag> [rounds]
export TMPDIR=/tmp
T=${1:-ab}; N=${2:-2}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/${T}.jsonl
for r in $(seq $N); do
  for v in base new; do
    if [ $v = base ]; then export TI_LIB=$GRAFT_REPO_ROOT/exp/base/libturboinfer_amd.so; else unset TI_LIB; fi
    timeout -k 10 200 python3 bench.py --batch 64 --steps 32 --warmup 4 --no-cpu-baseline | sed "s/^/$v c3 /" >> gpurun_out/${T}.jsonl || exit 1
    timeout -k 10 200 python3 bench.py --model llama3-8b --batch 32 --kv 8192 --steps 32 --warmup 4 --no-cpu-baseline | sed "s/^/$v c4 /" >> gpurun_out/${T}.jsonl || exit 1
  done
done
