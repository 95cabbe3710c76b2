#!/bin/bash
# Persistent decode (TI_PDS=1) A/B on one box: product (AHEAD 3, thinned loader) vs AHEAD 2 (pa2)
# vs no thinning during gathers (pnothin); the graph path between them as the reference.
# exp/<v>/ built with `make BUILD=exp/b_<v> LIB=exp/<v>/libturboinfer_amd.so EXTRA=-D...`.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r4_pds_ab.txt
for v in graph base pa2 pnothin base graph; do
  L=""; P=1
  [ $v = graph ] && P=0
  [ $v = pa2 ] || [ $v = pnothin ] && L=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so
  TI_PDS=$P TI_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/pab_$v.json 2>> gpurun_out/r4_pds_ab.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/pab_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'), d.get('calibration'))")" >> gpurun_out/r4_pds_ab.txt
done
