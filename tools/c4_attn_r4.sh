#!/bin/bash
# configs[4] attention (32 streams x 8 kv-heads x 8192 keys, one workgroup per CU): product
# (8 waves, ring 4) vs a per-workgroup rotated sweep start (rot), 16 waves with ring 2 (w16r2)
# and both (w16r2rot); exp/<v>/ built with `make BUILD=exp/b_<v> LIB=exp/<v>/... EXTRA=-D...`.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/c4_attn_r4.txt
for v in base rot w16r2 w16r2rot base rot; do
  if [ $v = base ]; then L=""; else L=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so; fi
  TI_LIB=$L timeout -k 10 300 python3 -u bench.py --model llama3-8b --batch 32 --kv 8192 --steps 16 --warmup 3 --no-cpu-baseline > gpurun_out/c4a_$v.json 2>> gpurun_out/c4_attn_r4.err
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/c4a_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('attention'))")" >> gpurun_out/c4_attn_r4.txt
done
for v in rot w16r2rot; do
  TI_LIB=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_engine.py -x -q -k "llama3 or 8192" --timeout 200 --timeout-method thread > gpurun_out/c4a_tests_$v.log 2>&1
done
