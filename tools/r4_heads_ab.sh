#!/bin/bash
# the driver's round-2 head (a0297c6, 741.8 tok/s) vs round-3 head (ed407dc,
# 711.3) vs HEAD, each with its own bench.py and library (git worktrees under exp/tree_<sha>),
# interleaved three times on one box with the driver's own command (minus the CPU baseline leg).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r4_heads_ab.txt
for round in 1 2 3; do
  for v in a0297c6 ed407dc HEAD; do
    if [ $v = HEAD ]; then d=$GRAFT_REPO_ROOT; else d=$GRAFT_REPO_ROOT/exp/tree_$v; fi
    (cd $d && timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline) > gpurun_out/hab_${v}_$round.json 2>> gpurun_out/r4_heads_ab.err || exit 1
    echo "$round $v $(python3 -c "import json;d=json.load(open('gpurun_out/hab_${v}_$round.json'));print(d['value'], d['ms_per_step'], d.get('calibration'))")" >> gpurun_out/r4_heads_ab.txt
  done
done
