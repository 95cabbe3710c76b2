#!/bin/bash
# configs[3] (64 x 7B @ 2048): attention split count (bench --attn-splits; 0 = the engine's policy).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c3splits
mkdir -p $O
for r in 1 2; do
  for sp in 0 2 3 4; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --kernel-reps 20 --steps 32 --warmup 4 --batch 64 --attn-splits $sp \
      > $O/s${sp}_$r.json 2> $O/s${sp}_$r.err || exit 1
    python3 -c "import json;d=json.load(open('$O/s${sp}_$r.json'));print('splits $sp',$r,d['value'],d['kernels']['attention']['avg_us'],d['kernels']['attention']['GBps'])"
  done
done
