#!/bin/bash
# Batched fold A/B (TI_FOLD=0 also turns the one-stream fold off, so only the batched configs are
# compared): configs[3] (7B, 64 streams, KV 2048) and configs[4] (Llama-3-8B, 32 streams, KV 8192),
# interleaved twice on one box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r4_fold_ab.txt
for r in 1 2; do
  for f in 1 0; do
    TI_FOLD=$f timeout -k 10 300 python3 -u bench.py --model llama2-7b --batch 64 --kv 2048 --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/fab_c3_$f.json 2>> gpurun_out/r4_fold_ab.err || exit 1
    TI_FOLD=$f timeout -k 10 300 python3 -u bench.py --model llama3-8b --batch 32 --kv 8192 --steps 16 --warmup 3 --no-cpu-baseline > gpurun_out/fab_c4_$f.json 2>> gpurun_out/r4_fold_ab.err || exit 1
    for c in c3 c4; do
      echo "$r fold=$f $c $(python3 -c "import json;d=json.load(open('gpurun_out/fab_${c}_$f.json'));k=d['kernels'];print(d['value'], d['ms_per_step'], {n:k[n]['avg_us'] for n in ('qkv','o','gate_up','down','lm_head','attention')})")" >> gpurun_out/r4_fold_ab.txt
    done
  done
done
