#!/bin/bash
# configs[4] (Llama-3-8B GQA, 32 streams, KV 8192): attention workgroup target A/B (TI_ATTN_TARGET).
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/c4_attn_ab.txt
for t in 256 512 1024 2048; do
  TI_ATTN_TARGET=$t timeout -k 10 300 python3 -u bench.py --model llama3-8b --batch 32 --kv 8192 --steps 16 --warmup 3 --no-cpu-baseline > gpurun_out/c4_t$t.json 2>> gpurun_out/c4_attn_ab.err
  echo "$t $(python3 -c "import json;d=json.load(open('gpurun_out/c4_t$t.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('attention'))")" >> gpurun_out/c4_attn_ab.txt
done
for t in 1024 2048; do
  TI_ATTN_TARGET=$t timeout -k 10 300 python3 -u bench.py --batch 64 --steps 16 --warmup 3 --no-cpu-baseline > gpurun_out/c3_t$t.json 2>> gpurun_out/c4_attn_ab.err
  echo "c3 $t $(python3 -c "import json;d=json.load(open('gpurun_out/c3_t$t.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('attention'))")" >> gpurun_out/c4_attn_ab.txt
done
