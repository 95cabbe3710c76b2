#!/bin/bash
# Persistent decode ring knobs on one box (7B bench, TI_PDS=1): product (thin during gathers,
# 3 fills ahead) vs no thinning (pt0), 4 ahead (pa4), 2 ahead (pa2), both (pt0a4); graph reference.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r4j_bench.txt
for v in base pt0 pa4 pa2 pt0a4 base graph; do
  L=""; P=1
  [ $v = graph ] && P=0
  case $v in base|graph) ;; *) L=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so;; esac
  TI_PDS=$P TI_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 60 --warmup 8 --no-cpu-baseline > gpurun_out/r4j_$v.json 2>> gpurun_out/r4j_bench.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r4j_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4j_bench.txt
done
echo "done10"
