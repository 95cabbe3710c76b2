#!/bin/bash
# Second round-4 GPU call: persistent-decode variant A/B, TinyLlama (configs[1]) graph vs persistent,
# then the round-head interleave.  Each step bounded; stops at the first failure.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/r4_pds_ab.sh || exit 1
echo "pds ab done"
: > gpurun_out/r4_tl.txt
for v in graph pds graph pds; do
  P=0; [ $v = pds ] && P=1
  TI_PDS=$P timeout -k 10 200 python3 -u bench.py --model tinyllama-1.1b --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/tl_$v.json 2>> gpurun_out/r4_tl.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/tl_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4_tl.txt
done
echo "tinyllama done"
bash tools/r4_heads_ab.sh || exit 1
echo "heads done"
